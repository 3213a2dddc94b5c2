// dora-gpu-runtime: a runtime node hosting shared-library operators — the counterpart of
// binaries/runtime (src/lib.rs:150-260, src/operator/shared_lib.rs:30-295).
//
//   DORA_GPU_OPERATORS="op1=/path/libop1.so|out1,out2;op2=/path/libop2.so"  (+ the node env)
//
// The node's inputs and outputs are named `<operator>/<id>`.  Each input event goes to its
// operator's dora_on_event as a RawEvent whose Input carries the array in host memory (a
// device sample is downloaded first: operators read their inputs on the CPU, as they read shm
// in the reference).  Every output an operator sends through its SendOutput closure is packed
// into a device sample of this node (dora_node_send_output with the host array: plan + H2D
// pack, shared_lib.rs:108-140) under `<operator>/<output>`, with the reference's
// `open_telemetry_context` parameter.  Stop goes to every operator; an operator returning
// DORA_STATUS_STOP has its outputs closed and is dropped; the runtime ends when none is left
// or the event stream closes.
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "dora_gpu.h"
#include "operator_rt.h"
#include "params.h"

namespace {

using InitFn = DoraInitResult_t (*)();
using DropFn = DoraResult_t (*)(void*);
using EventFn = OnEventResult_t (*)(RawEvent_t*, const SendOutput_t*, void*);

struct Operator {
  std::string id;
  bool host_only = false;  // the node has no GPU (DORA_GPU_DEVICE < 0)
  void* lib = nullptr;
  InitFn init = nullptr;
  DropFn drop = nullptr;
  EventFn on_event = nullptr;
  void* context = nullptr;
  bool running = false;
  dora_node* node = nullptr;
  std::vector<std::string> outputs;  // full ids `<operator>/<output>`: declared + sent
};

std::string take_error(DoraResult_t r) {
  if (!r.error) return {};
  std::string m(reinterpret_cast<const char*>(r.error->ptr), r.error->len);
  std::free(r.error->ptr);
  std::free(r.error);
  return m.empty() ? "unknown error" : m;
}

Vec_uint8_t borrowed(const std::string& s) {
  // a view of `s` (NUL-terminated after len) valid for the duration of the call
  return Vec_uint8_t{reinterpret_cast<uint8_t*>(const_cast<char*>(s.c_str())), s.size(), s.size()};
}

// SendOutput::call — one operator output into a device sample of this node.
DoraResult_t send_output_call(void* env, Output_t out) {
  auto* op = static_cast<Operator*>(env);
  std::string id = op->id + "/" + (out.id ? out.id : "");
  std::free(out.id);
  std::map<std::string, Param> params;
  params["open_telemetry_context"] = Param{2, 0, ""};
  const std::vector<uint8_t> enc = encode_params(params);
  int rc = dora_node_send_output(op->node, id.c_str(), &out.array, &out.schema, ARROW_DEVICE_CPU,
                                 enc.data(), enc.size());
  // the host array may go once the copy into the sample has completed (a host-only node copied
  // it into an inline sample already)
  if (rc == DORA_OK && !op->host_only) rc = dora_gpu_stream_sync(dora_node_stream(op->node));
  std::string err = rc == DORA_OK ? "" : dora_gpu_last_error();
  if (out.array.release) out.array.release(&out.array);
  if (out.schema.release) out.schema.release(&out.schema);
  if (rc != DORA_OK) return dora_operator_error(("failed to send output `" + id + "`: " + err).c_str());
  bool known = false;
  for (auto& o : op->outputs) known |= o == id;
  if (!known) op->outputs.push_back(id);
  return DoraResult_t{nullptr};
}

void noop(void*) {}

// The input of an event as a host array owned by `in`.
int input_array(dora_event* ev, Input* in) {
  ArrowArray a{};
  ArrowSchema s{};
  int rc = dora_event_array(ev, &a, &s);
  if (rc != DORA_OK) return rc;
  if (!dora_event_is_device(ev)) {
    in->array = a;  // host Vec sample, imported in place
    in->schema = s;
    return DORA_OK;
  }
  ArrowArray h{};
  rc = dora_gpu_array_download(&a, &s, &h);
  if (a.release) a.release(&a);
  if (rc != DORA_OK) {
    if (s.release) s.release(&s);
    return rc;
  }
  in->array = h;
  in->schema = s;
  return DORA_OK;
}

int fail_op(Operator& op, const char* what, const std::string& msg) {
  std::fprintf(stderr, "runtime: operator `%s` %s: %s\n", op.id.c_str(), what, msg.c_str());
  return 1;
}

void stop_operator(Operator& op) {
  if (!op.running) return;
  op.running = false;
  if (!op.outputs.empty()) {
    std::vector<const char*> ids;
    for (auto& o : op.outputs) ids.push_back(o.c_str());
    (void)dora_node_close_outputs(op.node, ids.data(), ids.size());
  }
  std::string e = take_error(op.drop(op.context));
  if (!e.empty()) std::fprintf(stderr, "runtime: dropping operator `%s`: %s\n", op.id.c_str(), e.c_str());
}

}  // namespace

int main() {
  const char* spec = std::getenv("DORA_GPU_OPERATORS");
  if (!spec || !*spec) {
    std::fprintf(stderr, "runtime: DORA_GPU_OPERATORS is not set\n");
    return 2;
  }
  std::vector<Operator> ops;
  {
    std::string s(spec);
    size_t at = 0;
    while (at <= s.size()) {
      size_t end = s.find(';', at);
      if (end == std::string::npos) end = s.size();
      std::string item = s.substr(at, end - at);
      at = end + 1;
      if (item.empty()) continue;
      const size_t eq = item.find('=');
      if (eq == std::string::npos) {
        std::fprintf(stderr, "runtime: bad operator spec `%s`\n", item.c_str());
        return 2;
      }
      Operator op;
      op.id = item.substr(0, eq);
      std::string path = item.substr(eq + 1);
      const size_t bar = path.find('|');
      if (bar != std::string::npos) {  // the operator's declared outputs (closed when it stops)
        std::string outs = path.substr(bar + 1);
        path.resize(bar);
        size_t k = 0;
        while (k < outs.size()) {
          size_t c = outs.find(',', k);
          if (c == std::string::npos) c = outs.size();
          if (c > k) op.outputs.push_back(op.id + "/" + outs.substr(k, c - k));
          k = c + 1;
        }
      }
      op.lib = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
      if (!op.lib) return fail_op(op, "failed to load", dlerror());
      op.init = reinterpret_cast<InitFn>(dlsym(op.lib, "dora_init_operator"));
      op.drop = reinterpret_cast<DropFn>(dlsym(op.lib, "dora_drop_operator"));
      op.on_event = reinterpret_cast<EventFn>(dlsym(op.lib, "dora_on_event"));
      if (!op.init || !op.drop || !op.on_event)
        return fail_op(op, "lacks an entry point", "dora_init_operator / dora_drop_operator / dora_on_event");
      ops.push_back(op);
    }
  }
  dora_node* node = nullptr;
  if (dora_node_init_from_env(&node) != DORA_OK) {
    std::fprintf(stderr, "runtime: init failed: %s\n", dora_gpu_last_error());
    return 1;
  }
  const char* dev = std::getenv("DORA_GPU_DEVICE");
  for (auto& op : ops) {
    op.node = node;
    op.host_only = dev && std::atoi(dev) < 0;
    DoraInitResult_t r = op.init();
    std::string e = take_error(r.result);
    if (!e.empty()) {
      dora_node_free(node);
      return fail_op(op, "init_operator failed", e);
    }
    op.context = r.operator_context;
    op.running = true;
  }
  int status = 0;
  auto deliver = [&](Operator& op, RawEvent_t* raw) {
    SendOutput_t send{{&op, send_output_call, noop, noop}};
    OnEventResult_t r = op.on_event(raw, &send, op.context);
    std::string e = take_error(r.result);
    if (!e.empty()) {
      status = fail_op(op, "on_event failed", e);
      return false;
    }
    if (r.status == DORA_STATUS_STOP) stop_operator(op);
    if (r.status == DORA_STATUS_STOP_ALL)
      for (auto& o : ops) stop_operator(o);
    return true;
  };
  auto running = [&] {
    for (auto& o : ops)
      if (o.running) return true;
    return false;
  };
  while (status == 0 && running()) {
    dora_event* ev = nullptr;
    int rc = dora_node_next_event(node, -1, &ev);
    if (rc == DORA_ERR_CLOSED) break;
    if (rc != DORA_OK) {
      std::fprintf(stderr, "runtime: next_event: %s\n", dora_gpu_last_error());
      status = 1;
      break;
    }
    const int type = dora_event_type(ev);
    const std::string full = dora_event_id(ev);
    const size_t slash = full.find('/');
    Operator* target = nullptr;
    if (slash != std::string::npos)
      for (auto& o : ops)
        if (o.running && full.compare(0, slash, o.id) == 0 && o.id.size() == slash) target = &o;
    const std::string local = slash == std::string::npos ? full : full.substr(slash + 1);
    if (type == DORA_EVENT_INPUT && target) {
      Input in;
      in.id = local;
      if (input_array(ev, &in) != DORA_OK) {
        std::fprintf(stderr, "runtime: input `%s`: %s\n", full.c_str(), dora_gpu_last_error());
        status = 1;
      } else {
        RawEvent_t raw{&in, {nullptr, 0, 0}, false, {nullptr, 0, 0}};
        deliver(*target, &raw);
      }
    } else if (type == DORA_EVENT_INPUT_CLOSED && target) {
      RawEvent_t raw{nullptr, borrowed(local), false, {nullptr, 0, 0}};
      deliver(*target, &raw);
    } else if (type == DORA_EVENT_STOP) {
      for (auto& o : ops) {
        if (!o.running) continue;
        RawEvent_t raw{nullptr, {nullptr, 0, 0}, true, {nullptr, 0, 0}};
        if (!deliver(o, &raw)) break;
      }
    } else if (type == DORA_EVENT_ERROR) {
      const std::string msg = dora_event_error(ev);
      for (auto& o : ops) {
        if (!o.running) continue;
        RawEvent_t raw{nullptr, {nullptr, 0, 0}, false, borrowed(msg)};
        if (!deliver(o, &raw)) break;
      }
    } else if (type == DORA_EVENT_ALL_INPUTS_CLOSED) {
      dora_event_free(ev);
      break;
    }
    dora_event_free(ev);
  }
  for (auto& o : ops) stop_operator(o);
  dora_node_free(node);
  // operator libraries stay loaded until exit: outputs they allocated may still be referenced
  return status;
}
