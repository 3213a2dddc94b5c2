// Helper functions of the shared-library operator ABI (include/dora_operator_api.h): the
// counterparts of `dora_read_input_id`, `dora_read_data`, `dora_send_operator_output` ... in
// apis/rust/operator/types/src/lib.rs:156-186, which the reference links into every operator.
#include <cstdlib>
#include <cstring>
#include <string>

#include "common.h"
#include "operator_rt.h"

namespace {

Vec_uint8_t vec_copy(const void* p, size_t n) {
  Vec_uint8_t v{nullptr, 0, 0};
  v.ptr = static_cast<uint8_t*>(std::malloc(n ? n : 1));
  if (!v.ptr) return v;
  if (n) std::memcpy(v.ptr, p, n);
  v.len = v.cap = n;
  return v;
}

// A one-buffer-pair UInt8 array owning a copy of `n` bytes (`Vec<u8>::into_arrow`).
struct BytesArray {
  const void* buffers[2];
  uint8_t* data;
};

void release_bytes_array(ArrowArray* a) {
  auto* p = static_cast<BytesArray*>(a->private_data);
  std::free(p->data);
  delete p;
  a->release = nullptr;
}

void release_u8_schema(ArrowSchema* s) { s->release = nullptr; }

DoraResult_t call_send(const SendOutput_t* send_output, const char* id, ArrowArray* array,
                       ArrowSchema* schema) {
  Output out;
  out.id = strdup(id);
  out.array = *array;
  out.schema = *schema;
  array->release = nullptr;  // moved into the output
  schema->release = nullptr;
  if (!out.id) {
    if (out.array.release) out.array.release(&out.array);
    if (out.schema.release) out.schema.release(&out.schema);
    return dora_operator_error("out of host memory");
  }
  return send_output->send_output.call(send_output->send_output.env_ptr, out);
}

}  // namespace

extern "C" {

char* dora_read_input_id(const Input_t* input) { return input ? strdup(input->id.c_str()) : nullptr; }

void dora_free_input_id(char* input_id) { std::free(input_id); }

Vec_uint8_t dora_read_data(Input_t* input) {
  Vec_uint8_t none{nullptr, 0, 0};
  if (!input || input->taken || !input->array.release) return none;
  input->taken = true;  // `data_array.take()`: a second read yields nothing
  const ArrowArray& a = input->array;
  // `TryFrom<&ArrowData> for &[u8]` (libraries/arrow-convert/src/from_impls.rs:146-157):
  // a UInt8 primitive array without nulls
  if (!input->schema.format || std::strcmp(input->schema.format, "C") != 0 || a.null_count != 0 ||
      a.n_buffers != 2)
    return none;
  const auto* values = static_cast<const uint8_t*>(a.buffers[1]);
  if (!values && a.length) return none;
  return vec_copy(values ? values + a.offset : nullptr, size_t(a.length));
}

void dora_free_data(Vec_uint8_t data) { std::free(data.ptr); }

DoraResult_t dora_send_operator_output(const SendOutput_t* send_output, const char* id,
                                       const uint8_t* data_ptr, size_t data_len) {
  if (!send_output || !id || (!data_ptr && data_len)) return dora_operator_error("NULL argument");
  auto* p = new BytesArray();
  p->data = static_cast<uint8_t*>(std::malloc(data_len ? data_len : 1));
  if (!p->data) {
    delete p;
    return dora_operator_error("out of host memory");
  }
  if (data_len) std::memcpy(p->data, data_ptr, data_len);
  p->buffers[0] = nullptr;
  p->buffers[1] = p->data;
  ArrowArray a{};
  a.length = int64_t(data_len);
  a.n_buffers = 2;
  a.buffers = p->buffers;
  a.release = release_bytes_array;
  a.private_data = p;
  ArrowSchema s{};
  s.format = "C";
  s.name = "";
  s.release = release_u8_schema;
  return call_send(send_output, id, &a, &s);
}

int dora_input_arrow(const Input_t* input, const ArrowArray** array, const ArrowSchema** schema) {
  if (!input || !array || !schema) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  if (!input->array.release) return dora::fail(DORA_ERR_INVALID, "input has no array");
  *array = &input->array;
  *schema = &input->schema;
  return DORA_OK;
}

DoraResult_t dora_send_operator_output_arrow(const SendOutput_t* send_output, const char* id,
                                             ArrowArray* array, ArrowSchema* schema) {
  if (!send_output || !id || !array || !schema) return dora_operator_error("NULL argument");
  return call_send(send_output, id, array, schema);
}

DoraResult_t dora_operator_error(const char* message) {
  DoraResult_t r{nullptr};
  const char* m = message ? message : "";
  auto* v = static_cast<Vec_uint8_t*>(std::malloc(sizeof(Vec_uint8_t)));
  if (!v) return r;
  *v = vec_copy(m, std::strlen(m));
  r.error = v;
  return r;
}

}  // extern "C"
