/* Shared-library operator ABI of the device data plane.
 *
 * The reference's C operator interface (apis/c/operator/operator_api.h, operator_types.h,
 * generated from apis/rust/operator/types/src/lib.rs:19-186): an operator library exports
 * dora_init_operator / dora_on_event / dora_drop_operator; `dora-gpu-runtime` loads it, hands
 * it RawEvents and a SendOutput closure, and packs every output it sends into a device sample
 * (binaries/runtime/src/operator/shared_lib.rs:108-140: required_data_size +
 * copy_array_into_sample, here dora_gpu_plan + the pack kernel).  The type names, field order
 * and entry points are the reference's, so an operator written against the reference header
 * builds against this one unchanged; Input and Output stay opaque as there.  The helper
 * functions below live in libdora_gpu.so (the reference links them into the operator from the
 * operator-api crate).
 */
#ifndef DORA_OPERATOR_API_H
#define DORA_OPERATOR_API_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DORA_OPERATOR_EXPORT __attribute__((visibility("default")))

struct ArrowArray;  /* Arrow C Data Interface (dora_gpu.h) */
struct ArrowSchema;

/* A byte vector owned by whoever the call says (safer_ffi::Vec<u8> layout); ptr NULL = none. */
typedef struct Vec_uint8 {
  uint8_t* ptr;
  size_t len;
  size_t cap;
} Vec_uint8_t;

/* error NULL: success; otherwise a boxed message (dora_operator_error builds one). */
typedef struct DoraResult {
  Vec_uint8_t* error;
} DoraResult_t;

typedef struct DoraInitResult {
  DoraResult_t result;
  void* operator_context;
} DoraInitResult_t;

enum DoraStatus {
  DORA_STATUS_CONTINUE = 0,
  DORA_STATUS_STOP = 1,
  DORA_STATUS_STOP_ALL = 2,
};
typedef uint8_t DoraStatus_t;

typedef struct OnEventResult {
  DoraResult_t result;
  DoraStatus_t status;
} OnEventResult_t;

typedef struct Input Input_t;   /* opaque: id, Arrow array (host), metadata */
typedef struct Output Output_t; /* opaque: id, Arrow array, metadata */

/* Exactly one of: an input, a closed input id, stop, an error (the others NULL / false). */
typedef struct RawEvent {
  Input_t* input;
  Vec_uint8_t input_closed;
  bool stop;
  Vec_uint8_t error;
} RawEvent_t;

typedef struct ArcDynFn1_DoraResult_Output {
  void* env_ptr;
  DoraResult_t (*call)(void*, Output_t);
  void (*release)(void*);
  void (*retain)(void*);
} ArcDynFn1_DoraResult_Output_t;

typedef struct SendOutput {
  ArcDynFn1_DoraResult_Output_t send_output;
} SendOutput_t;

typedef struct Metadata {
  Vec_uint8_t open_telemetry_context;
} Metadata_t;

/* Entry points an operator library exports (implemented by the operator, not by this library). */
DORA_OPERATOR_EXPORT DoraInitResult_t dora_init_operator(void);
DORA_OPERATOR_EXPORT DoraResult_t dora_drop_operator(void* operator_context);
DORA_OPERATOR_EXPORT OnEventResult_t dora_on_event(RawEvent_t* event,
                                                   const SendOutput_t* send_output,
                                                   void* operator_context);

/* Helpers (libdora_gpu.so), as in the reference's operator-api crate (types/src/lib.rs:156-186).
 * dora_read_input_id: a malloc'ed copy of the input id (free with dora_free_input_id).
 * dora_read_data: the bytes of a UInt8 input without nulls, copied (free with dora_free_data);
 *   ptr NULL for any other input or when called twice (the array is taken, lib.rs:165-171).
 * dora_send_operator_output: send `data_len` bytes as a UInt8 array on output `id`. */
char* dora_read_input_id(const Input_t* input);
void dora_free_input_id(char* input_id);
Vec_uint8_t dora_read_data(Input_t* input);
void dora_free_data(Vec_uint8_t data);
DoraResult_t dora_send_operator_output(const SendOutput_t* send_output, const char* id,
                                       const uint8_t* data_ptr, size_t data_len);

/* Extensions of this build (no reference counterpart): the input as an Arrow C Data Interface
 * array in host memory (the operator may read it until the event ends; ownership stays with the
 * input), an output from any Arrow array (moved: the call releases it), and an error result. */
int dora_input_arrow(const Input_t* input, const struct ArrowArray** array,
                     const struct ArrowSchema** schema);
DoraResult_t dora_send_operator_output_arrow(const SendOutput_t* send_output, const char* id,
                                             struct ArrowArray* array, struct ArrowSchema* schema);
DoraResult_t dora_operator_error(const char* message);

#ifdef __cplusplus
}
#endif

#endif /* DORA_OPERATOR_API_H */
