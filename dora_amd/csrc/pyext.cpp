// dora_amd._dora_node: the per-send hot path of the Python node API as a CPython extension.
//
// The reference's Python node is a native extension too (PyO3: apis/python/node/src/lib.rs:
// 157-185 `send_output`, whose metadata goes through pydict_to_metadata,
// apis/python/operator/src/lib.rs:165-186).  Through ctypes a send paid ~1 us encoding the
// parameters in Python and ~0.9 us of ctypes argument conversion; here both are one METH_FASTCALL
// call.  The GIL is released around the library call: a send may wait for drop tokens that
// another Python thread of the same process returns.
//
// The receive side likewise: next_event returns an event's fields and decoded parameters in one
// call (the reference: PyO3 `Node.next` -> PyEvent, apis/python/node/src/lib.rs:89-108), instead
// of ~8 ctypes calls and a Python decode (30 us per inline 8-byte input through ctypes).
//
// Every function returns the library's status code; dora_amd/node.py raises on non-zero (the
// message comes from dora_gpu_last_error), so error behaviour is the ctypes path's.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <time.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>

#include "dora_gpu.h"

namespace {

void put_u32(std::string& o, uint32_t v) { o.append(reinterpret_cast<const char*>(&v), 4); }
void put_u64(std::string& o, uint64_t v) { o.append(reinterpret_cast<const char*>(&v), 8); }

// MetadataParameters encoding (include/dora_gpu.h, dora_node_send_output_sample): u32 count,
// then per entry in sorted key order: u64 key length, key, u8 tag (0 bool, 1 int, 2 string),
// value (u8 | i64 | u64 length + utf-8).  Anything else is stringified (str(v)), as
// pydict_to_metadata does.  Same bytes as dora_amd.node.encode_parameters_py.
bool encode(PyObject* meta, std::string& out) {
  out.clear();
  if (meta == nullptr || meta == Py_None) return true;
  if (!PyDict_Check(meta)) {
    PyErr_SetString(PyExc_TypeError, "metadata must be a dict or None");
    return false;
  }
  if (PyDict_GET_SIZE(meta) == 0) return true;
  PyObject* keys = PyDict_Keys(meta);
  if (!keys) return false;
  if (PyList_Sort(keys) < 0) {
    Py_DECREF(keys);
    return false;
  }
  const Py_ssize_t n = PyList_GET_SIZE(keys);
  put_u32(out, uint32_t(n));
  bool ok = true;
  for (Py_ssize_t i = 0; ok && i < n; ++i) {
    PyObject* k = PyList_GET_ITEM(keys, i);
    PyObject* ks = PyUnicode_Check(k) ? (Py_INCREF(k), k) : PyObject_Str(k);
    if (!ks) {
      ok = false;
      break;
    }
    Py_ssize_t kl = 0;
    const char* kb = PyUnicode_AsUTF8AndSize(ks, &kl);
    if (!kb) {
      Py_DECREF(ks);
      ok = false;
      break;
    }
    put_u64(out, uint64_t(kl));
    out.append(kb, size_t(kl));
    Py_DECREF(ks);
    PyObject* v = PyDict_GetItemWithError(meta, k);  // borrowed
    if (!v) {
      ok = false;
      break;
    }
    if (PyBool_Check(v)) {
      out.push_back(char(0));
      out.push_back(char(v == Py_True ? 1 : 0));
    } else if (PyLong_Check(v)) {
      const long long x = PyLong_AsLongLong(v);
      if (x == -1 && PyErr_Occurred()) {
        ok = false;  // OverflowError, as struct.pack("<q") raises
        break;
      }
      out.push_back(char(1));
      put_u64(out, uint64_t(x));
    } else {
      PyObject* s = PyUnicode_Check(v) ? (Py_INCREF(v), v) : PyObject_Str(v);
      if (!s) {
        ok = false;
        break;
      }
      Py_ssize_t sl = 0;
      const char* sb = PyUnicode_AsUTF8AndSize(s, &sl);
      if (!sb) {
        Py_DECREF(s);
        ok = false;
        break;
      }
      out.push_back(char(2));
      put_u64(out, uint64_t(sl));
      out.append(sb, size_t(sl));
      Py_DECREF(s);
    }
  }
  Py_DECREF(keys);
  return ok;
}

thread_local std::string t_params;

bool as_ptr(PyObject* o, void** p) {
  if (o == Py_None) {
    *p = nullptr;
    return true;
  }
  *p = PyLong_AsVoidPtr(o);
  return !(*p == nullptr && PyErr_Occurred());
}

const char* as_cstr(PyObject* o) {
  if (PyBytes_Check(o)) return PyBytes_AS_STRING(o);
  if (PyUnicode_Check(o)) return PyUnicode_AsUTF8(o);
  PyErr_SetString(PyExc_TypeError, "output id must be str or bytes");
  return nullptr;
}

PyObject* py_encode_parameters(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 1) {
    PyErr_SetString(PyExc_TypeError, "encode_parameters(metadata)");
    return nullptr;
  }
  if (!encode(args[0], t_params)) return nullptr;
  return PyBytes_FromStringAndSize(t_params.data(), Py_ssize_t(t_params.size()));
}

// Optional trailing `flags` argument (DORA_SEND_ASYNC) of send_bytes / send_array.
bool send_flags(PyObject* const* args, Py_ssize_t nargs, uint32_t* flags) {
  *flags = 0;
  if (nargs < 7) return true;
  const unsigned long f = PyLong_AsUnsignedLong(args[6]);
  if (f == static_cast<unsigned long>(-1) && PyErr_Occurred()) return false;
  *flags = static_cast<uint32_t>(f);
  return true;
}

// send_bytes(handle, output_id, data_ptr, len, device_type, metadata[, flags]) -> status
PyObject* py_send_bytes(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 6 && nargs != 7) {
    PyErr_SetString(PyExc_TypeError,
                    "send_bytes(handle, output_id, data_ptr, len, device_type, metadata[, flags])");
    return nullptr;
  }
  uint32_t flags = 0;
  if (!send_flags(args, nargs, &flags)) return nullptr;
  void *h = nullptr, *data = nullptr;
  if (!as_ptr(args[0], &h) || !as_ptr(args[2], &data)) return nullptr;
  const char* oid = as_cstr(args[1]);
  if (!oid) return nullptr;
  const size_t len = PyLong_AsSize_t(args[3]);
  if (len == size_t(-1) && PyErr_Occurred()) return nullptr;
  const long dev = PyLong_AsLong(args[4]);
  if (dev == -1 && PyErr_Occurred()) return nullptr;
  std::string& params = t_params;
  if (!encode(args[5], params)) return nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = dora_node_send_output_bytes_ex(static_cast<dora_node*>(h), oid, data, len,
                                      static_cast<ArrowDeviceType>(dev),
                                      reinterpret_cast<const uint8_t*>(params.data()),
                                      params.size(), flags);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

// send_buffer(handle, output_id, buffer, metadata) -> status: host bytes (any object with the
// buffer protocol: bytes, bytearray, memoryview, numpy) as send_output_bytes of a host source,
// read in place — the call copies them (inline below 4096 B, else into a slot) before it returns
PyObject* py_send_buffer(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 4) {
    PyErr_SetString(PyExc_TypeError, "send_buffer(handle, output_id, buffer, metadata)");
    return nullptr;
  }
  void* h = nullptr;
  if (!as_ptr(args[0], &h)) return nullptr;
  const char* oid = as_cstr(args[1]);
  if (!oid) return nullptr;
  Py_buffer view;
  if (PyObject_GetBuffer(args[2], &view, PyBUF_C_CONTIGUOUS) != 0) return nullptr;
  std::string& params = t_params;
  if (!encode(args[3], params)) {
    PyBuffer_Release(&view);
    return nullptr;
  }
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = dora_node_send_output_bytes_ex(static_cast<dora_node*>(h), oid, view.buf,
                                      static_cast<size_t>(view.len), ARROW_DEVICE_CPU,
                                      reinterpret_cast<const uint8_t*>(params.data()),
                                      params.size(), 0);
  Py_END_ALLOW_THREADS
  PyBuffer_Release(&view);
  return PyLong_FromLong(rc);
}

// send_array(handle, output_id, array_addr, schema_addr, device_type, metadata[, flags])
PyObject* py_send_array(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 6 && nargs != 7) {
    PyErr_SetString(PyExc_TypeError, "send_array(handle, output_id, array_addr, schema_addr, "
                                     "device_type, metadata[, flags])");
    return nullptr;
  }
  uint32_t flags = 0;
  if (!send_flags(args, nargs, &flags)) return nullptr;
  void *h = nullptr, *arr = nullptr, *sch = nullptr;
  if (!as_ptr(args[0], &h) || !as_ptr(args[2], &arr) || !as_ptr(args[3], &sch)) return nullptr;
  const char* oid = as_cstr(args[1]);
  if (!oid) return nullptr;
  const long dev = PyLong_AsLong(args[4]);
  if (dev == -1 && PyErr_Occurred()) return nullptr;
  std::string& params = t_params;
  if (!encode(args[5], params)) return nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = dora_node_send_output_ex(static_cast<dora_node*>(h), oid,
                                static_cast<const struct ArrowArray*>(arr),
                                static_cast<const struct ArrowSchema*>(sch),
                                static_cast<ArrowDeviceType>(dev),
                                reinterpret_cast<const uint8_t*>(params.data()), params.size(),
                                flags);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

// MetadataParameters bytes -> dict (the inverse of encode; dora_amd.node.decode_parameters).
PyObject* decode(const uint8_t* p, size_t n) {
  PyObject* out = PyDict_New();
  if (!out || n < 4) return out;
  auto rd = [&](size_t at, size_t w, void* v) {
    if (at + w > n) return false;
    std::memcpy(v, p + at, w);
    return true;
  };
  uint32_t count = 0;
  rd(0, 4, &count);
  size_t i = 4;
  for (uint32_t e = 0; e < count; ++e) {
    uint64_t kl = 0;
    if (!rd(i, 8, &kl) || kl > n - i - 8) goto bad;
    i += 8;
    {
      PyObject* key = PyUnicode_DecodeUTF8(reinterpret_cast<const char*>(p + i), Py_ssize_t(kl), nullptr);
      if (!key) goto fail;
      i += kl;
      PyObject* val = nullptr;
      if (i >= n) {
        Py_DECREF(key);
        goto bad;
      }
      const uint8_t tag = p[i++];
      if (tag == 0) {
        if (i >= n) {
          Py_DECREF(key);
          goto bad;
        }
        val = PyBool_FromLong(p[i++] != 0);
      } else if (tag == 1) {
        int64_t x = 0;
        if (!rd(i, 8, &x)) {
          Py_DECREF(key);
          goto bad;
        }
        i += 8;
        val = PyLong_FromLongLong(x);
      } else {
        uint64_t sl = 0;
        if (!rd(i, 8, &sl) || sl > n - i - 8) {
          Py_DECREF(key);
          goto bad;
        }
        i += 8;
        val = PyUnicode_DecodeUTF8(reinterpret_cast<const char*>(p + i), Py_ssize_t(sl), nullptr);
        i += sl;
      }
      if (!val) {
        Py_DECREF(key);
        goto fail;
      }
      const int rc = PyDict_SetItem(out, key, val);
      Py_DECREF(key);
      Py_DECREF(val);
      if (rc < 0) goto fail;
    }
  }
  return out;
bad:
  PyErr_SetString(PyExc_ValueError, "truncated metadata parameters");
fail:
  Py_DECREF(out);
  return nullptr;
}

PyObject* params_of(const dora_event* ev) {
  const uint8_t* p = nullptr;
  size_t n = 0;
  if (dora_event_parameters(ev, &p, &n) != 0) return PyDict_New();
  return decode(p, n);
}

// next_event(handle, timeout_us) -> status (int) | (event_ptr, type, id, parameters, timestamp_ns,
// data_ptr, data_len, on_device, error).  The caller owns event_ptr (dora_event_free).  Inputs
// carry their decoded parameters; other events None.
PyObject* py_next_event(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2) {
    PyErr_SetString(PyExc_TypeError, "next_event(handle, timeout_us)");
    return nullptr;
  }
  void* h = nullptr;
  if (!as_ptr(args[0], &h)) return nullptr;
  const long long timeout = PyLong_AsLongLong(args[1]);
  if (timeout == -1 && PyErr_Occurred()) return nullptr;
  dora_event* ev = nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = dora_node_next_event(static_cast<dora_node*>(h), timeout, &ev);
  Py_END_ALLOW_THREADS
  if (rc != 0) return PyLong_FromLong(rc);
  const int type = dora_event_type(ev);
  PyObject* params = nullptr;
  const void* dp = nullptr;
  size_t dn = 0;
  int dev = 0;
  if (type == DORA_EVENT_INPUT) {
    params = params_of(ev);
    if (!params) {
      dora_event_free(ev);
      return nullptr;
    }
    // the data's address (a device input's mapping is opened here); its failure is the call's
    const int drc = dora_event_data(ev, &dp, &dn);
    if (drc != 0) {
      Py_DECREF(params);
      dora_event_free(ev);
      return PyLong_FromLong(drc);
    }
    dev = dora_event_is_device(ev);
  } else {
    Py_INCREF(Py_None);
    params = Py_None;
  }
  const char* err = type == DORA_EVENT_ERROR ? dora_event_error(ev) : "";
  PyObject* out =
      Py_BuildValue("(KisNKKnis)", static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(ev)),
                    type, dora_event_id(ev), params,
                    static_cast<unsigned long long>(dora_event_timestamp_ns(ev)),
                    static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(dp)),
                    static_cast<Py_ssize_t>(dn), dev, err);
  if (!out) dora_event_free(ev);  // (an id or error that is not UTF-8)
  return out;
}

// wait_input(handle, input_id, key, value, timeout_us) -> status (int) | parameters: the next
// input on `input_id` whose parameters have key == value; other events are consumed and freed.
PyObject* py_wait_input(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 5) {
    PyErr_SetString(PyExc_TypeError, "wait_input(handle, input_id, key, value, timeout_us)");
    return nullptr;
  }
  void* h = nullptr;
  if (!as_ptr(args[0], &h)) return nullptr;
  const char* want = as_cstr(args[1]);
  if (!want) return nullptr;
  long long left = PyLong_AsLongLong(args[4]);
  if (left == -1 && PyErr_Occurred()) return nullptr;
  const std::string want_id(want);
  PyObject* key = args[2];
  PyObject* value = args[3];
  for (;;) {
    dora_event* ev = nullptr;
    int rc;
    uint64_t t0 = 0, t1 = 0;
    Py_BEGIN_ALLOW_THREADS
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    t0 = uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
    rc = dora_node_next_event(static_cast<dora_node*>(h), left, &ev);
    clock_gettime(CLOCK_MONOTONIC, &ts);
    t1 = uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
    Py_END_ALLOW_THREADS
    if (rc != 0) return PyLong_FromLong(rc);
    left -= static_cast<long long>((t1 - t0) / 1000);
    if (dora_event_type(ev) == DORA_EVENT_INPUT && want_id == dora_event_id(ev)) {
      PyObject* params = params_of(ev);
      if (!params) {
        dora_event_free(ev);
        return nullptr;
      }
      PyObject* v = PyDict_GetItemWithError(params, key);  // borrowed
      const int eq = v ? PyObject_RichCompareBool(v, value, Py_EQ) : (PyErr_Occurred() ? -1 : 0);
      dora_event_free(ev);
      if (eq < 0) {
        Py_DECREF(params);
        return nullptr;
      }
      if (eq) return params;
      Py_DECREF(params);
    } else {
      dora_event_free(ev);
    }
    if (left <= 0) return PyLong_FromLong(DORA_ERR_TIMEOUT);
  }
}

// A pyarrow type's exported ArrowSchema, kept: a send lends it (dora_node_send_output borrows
// the schema), so a node sending arrays of one type exports each array only, not its type again
// (~3 us for a struct).  Looked up by the type object itself first, then by equality (a new
// array of an equal type) confirmed with field metadata (DataType.__eq__ ignores it, the
// serialized type keeps it); at most 64 types are kept.
void free_schema_capsule(PyObject* cap) {
  auto* s = static_cast<ArrowSchema*>(PyCapsule_GetPointer(cap, "dora_schema"));
  if (s && s->release) s->release(s);
  std::free(s);
}

PyObject* g_schemas = nullptr;   // type -> (type, capsule)
PyObject* g_last_type = nullptr;  // the last type sent and its capsule (strong references)
PyObject* g_last_cap = nullptr;

// A new reference to the capsule of `type`'s schema.  The caller keeps it for as long as the
// schema is in use (a send releases the GIL: another thread may evict the entry meanwhile).
PyObject* schema_for(PyObject* type) {
  if (type == g_last_type) {
    Py_INCREF(g_last_cap);
    return g_last_cap;
  }
  if (!g_schemas && !(g_schemas = PyDict_New())) return nullptr;
  PyObject* cap = nullptr;
  PyObject* hit = PyDict_GetItemWithError(g_schemas, type);  // borrowed (type, capsule)
  if (!hit && PyErr_Occurred()) return nullptr;
  if (hit) {
    // a strong reference for the call into Python below: code there may release the GIL, and
    // another sending thread may then clear g_schemas or replace this entry
    Py_INCREF(hit);
    PyObject* key = PyTuple_GET_ITEM(hit, 0);
    int same = key == type;
    if (!same) {
      // type.equals(key, check_metadata=True)
      static PyObject* kw = Py_BuildValue("{s:O}", "check_metadata", Py_True);
      PyObject* eq = kw ? PyObject_GetAttrString(type, "equals") : nullptr;
      PyObject* a = eq ? PyTuple_Pack(1, key) : nullptr;
      PyObject* r = a ? PyObject_Call(eq, a, kw) : nullptr;
      Py_XDECREF(a);
      Py_XDECREF(eq);
      if (!r) {
        Py_DECREF(hit);
        return nullptr;
      }
      same = PyObject_IsTrue(r);
      Py_DECREF(r);
      if (same < 0) {
        Py_DECREF(hit);
        return nullptr;
      }
    }
    if (same) {
      cap = PyTuple_GET_ITEM(hit, 1);
      Py_INCREF(cap);
    }
    Py_DECREF(hit);
  }
  if (!cap) {  // export it (replacing an entry equal but for field metadata)
    if (PyDict_GET_SIZE(g_schemas) >= 64) PyDict_Clear(g_schemas);
    auto* sc = static_cast<ArrowSchema*>(std::calloc(1, sizeof(ArrowSchema)));
    if (!sc) return PyErr_NoMemory();
    PyObject* r = PyObject_CallMethod(type, "_export_to_c", "K",
                                      static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(sc)));
    if (!r) {
      std::free(sc);
      return nullptr;
    }
    Py_DECREF(r);
    cap = PyCapsule_New(sc, "dora_schema", free_schema_capsule);
    if (!cap) {
      if (sc->release) sc->release(sc);
      std::free(sc);
      return nullptr;
    }
    PyObject* entry = PyTuple_Pack(2, type, cap);
    if (!entry || PyDict_SetItem(g_schemas, type, entry) < 0) {
      Py_XDECREF(entry);
      Py_DECREF(cap);
      return nullptr;
    }
    Py_DECREF(entry);
  }
  Py_INCREF(type);
  Py_XSETREF(g_last_type, type);
  Py_INCREF(cap);
  Py_XSETREF(g_last_cap, cap);
  return cap;
}

// send_pyarrow(handle, output_id, array, metadata) -> status: a host pyarrow.Array, exported
// (its type's schema from schema_for) and sent as dora_node_send_output of a host source, which
// copies it before returning (apis/python/node/src/lib.rs:157-185 -> arrow_utils.rs:23-71).
PyObject* py_send_pyarrow(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 4) {
    PyErr_SetString(PyExc_TypeError, "send_pyarrow(handle, output_id, array, metadata)");
    return nullptr;
  }
  void* h = nullptr;
  if (!as_ptr(args[0], &h)) return nullptr;
  const char* oid = as_cstr(args[1]);
  if (!oid) return nullptr;
  PyObject* type = PyObject_GetAttrString(args[2], "type");
  if (!type) return nullptr;
  PyObject* cap = schema_for(type);
  Py_DECREF(type);
  if (!cap) return nullptr;
  auto* schema = static_cast<ArrowSchema*>(PyCapsule_GetPointer(cap, "dora_schema"));
  std::string& params = t_params;
  ArrowArray a{};
  PyObject* r = encode(args[3], params) && schema
                    ? PyObject_CallMethod(args[2], "_export_to_c", "K",
                                          static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(&a)))
                    : nullptr;
  if (!r) {
    Py_DECREF(cap);
    return nullptr;
  }
  Py_DECREF(r);
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = dora_node_send_output_ex(static_cast<dora_node*>(h), oid, &a, schema, ARROW_DEVICE_CPU,
                                reinterpret_cast<const uint8_t*>(params.data()), params.size(), 0);
  Py_END_ALLOW_THREADS
  if (a.release) a.release(&a);
  Py_DECREF(cap);
  return PyLong_FromLong(rc);
}

// export_array(event_ptr) -> status (int) | (array_addr, schema_addr): the input's Arrow C
// structs (dora_event_array) in memory of this module, for pyarrow's _import_from_c, which moves
// their contents out; free_arrow(array_addr, schema_addr) then releases what is left and frees
// them (one native call each instead of two ctypes structures and a ctypes call).
PyObject* py_export_array(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 1) {
    PyErr_SetString(PyExc_TypeError, "export_array(event_ptr)");
    return nullptr;
  }
  void* ev = nullptr;
  if (!as_ptr(args[0], &ev)) return nullptr;
  auto* a = static_cast<ArrowArray*>(std::calloc(1, sizeof(ArrowArray)));
  auto* s = static_cast<ArrowSchema*>(std::calloc(1, sizeof(ArrowSchema)));
  if (!a || !s) {
    std::free(a);
    std::free(s);
    return PyErr_NoMemory();
  }
  const int rc = dora_event_array(static_cast<const dora_event*>(ev), a, s);
  if (rc != 0) {
    std::free(a);
    std::free(s);
    return PyLong_FromLong(rc);
  }
  return Py_BuildValue("(KK)", static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(a)),
                       static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(s)));
}

// A schema's identity as bytes: format, name, flags, metadata and children, recursively.
void schema_key(const ArrowSchema* s, std::string& k) {
  k += s->format ? s->format : "";
  k.push_back('\0');
  k += s->name ? s->name : "";
  k.push_back('\0');
  put_u64(k, uint64_t(s->flags));
  if (s->metadata) {  // int32 count, then per pair int32 length + bytes, twice
    const char* m = s->metadata;
    int32_t n = 0;
    std::memcpy(&n, m, 4);
    size_t len = 4;
    for (int32_t i = 0; i < 2 * n; ++i) {
      int32_t l = 0;
      std::memcpy(&l, m + len, 4);
      len += 4 + size_t(l);
    }
    put_u64(k, len);
    k.append(m, len);
  } else {
    put_u64(k, 0);
  }
  put_u64(k, uint64_t(s->n_children));
  for (int64_t i = 0; i < s->n_children; ++i) schema_key(s->children[i], k);
  k.push_back(s->dictionary ? 'D' : 'N');
  if (s->dictionary) schema_key(s->dictionary, k);
}

PyObject* g_types = nullptr;     // schema key -> pyarrow.DataType
PyObject* g_pa_dtype = nullptr;  // pyarrow.DataType

// export_typed(event_ptr) -> status (int) | (array_addr, pyarrow.DataType): as export_array, but
// the input's type comes from a cache keyed by its schema (pyarrow imports a schema in ~1-1.4 us
// per event; Array._import_from_c takes the DataType instead).  free_arrow(array_addr, 0) after
// the import.
PyObject* py_export_typed(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 1) {
    PyErr_SetString(PyExc_TypeError, "export_typed(event_ptr)");
    return nullptr;
  }
  void* ev = nullptr;
  if (!as_ptr(args[0], &ev)) return nullptr;
  if (!g_pa_dtype) {
    PyObject* pa = PyImport_ImportModule("pyarrow");
    if (!pa) return nullptr;
    g_pa_dtype = PyObject_GetAttrString(pa, "DataType");
    Py_DECREF(pa);
    if (!g_pa_dtype) return nullptr;
  }
  if (!g_types && !(g_types = PyDict_New())) return nullptr;
  auto* a = static_cast<ArrowArray*>(std::calloc(1, sizeof(ArrowArray)));
  ArrowSchema s{};
  if (!a) return PyErr_NoMemory();
  const int rc = dora_event_array(static_cast<const dora_event*>(ev), a, &s);
  if (rc != 0) {
    std::free(a);
    return PyLong_FromLong(rc);
  }
  std::string key;
  schema_key(&s, key);
  PyObject* kb = PyBytes_FromStringAndSize(key.data(), Py_ssize_t(key.size()));
  PyObject* dtype = kb ? PyDict_GetItemWithError(g_types, kb) : nullptr;  // borrowed
  if (dtype) {
    Py_INCREF(dtype);
  } else if (kb && !PyErr_Occurred()) {
    dtype = PyObject_CallMethod(g_pa_dtype, "_import_from_c", "K",
                                static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(&s)));
    if (dtype) {
      if (PyDict_GET_SIZE(g_types) >= 256) PyDict_Clear(g_types);
      if (PyDict_SetItem(g_types, kb, dtype) < 0) Py_CLEAR(dtype);
    }
  }
  Py_XDECREF(kb);
  if (s.release) s.release(&s);  // (moved out when pyarrow imported it)
  if (!dtype) {
    if (a->release) a->release(a);
    std::free(a);
    return nullptr;
  }
  return Py_BuildValue("(KN)", static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(a)),
                       dtype);
}

PyObject* py_free_arrow(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2) {
    PyErr_SetString(PyExc_TypeError, "free_arrow(array_addr, schema_addr)");
    return nullptr;
  }
  void *a = nullptr, *s = nullptr;
  if (!as_ptr(args[0], &a) || !as_ptr(args[1], &s)) return nullptr;
  auto* arr = static_cast<ArrowArray*>(a);
  auto* sch = static_cast<ArrowSchema*>(s);
  if (arr && arr->release) arr->release(arr);  // not imported (an error before the move)
  if (sch && sch->release) sch->release(sch);
  std::free(arr);
  std::free(sch);
  Py_RETURN_NONE;
}

PyMethodDef methods[] = {
    {"send_pyarrow", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(py_send_pyarrow)),
     METH_FASTCALL, "dora_node_send_output of a host pyarrow.Array (its type's schema kept)."},
    {"export_array", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(py_export_array)),
     METH_FASTCALL, "An input's Arrow C structs (dora_event_array), for pyarrow's _import_from_c."},
    {"export_typed", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(py_export_typed)),
     METH_FASTCALL, "An input's ArrowArray and its pyarrow.DataType (cached by schema)."},
    {"free_arrow", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(py_free_arrow)),
     METH_FASTCALL, "Release what is left of export_array's structs and free them."},
    {"next_event", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(py_next_event)),
     METH_FASTCALL, "dora_node_next_event with the event's fields and decoded parameters."},
    {"wait_input", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(py_wait_input)),
     METH_FASTCALL, "The next input on an id whose parameters have key == value."},
    {"encode_parameters", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(py_encode_parameters)),
     METH_FASTCALL, "MetadataParameters bytes of a dict (bool / int / str, else str(v))."},
    {"send_bytes", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(py_send_bytes)),
     METH_FASTCALL, "dora_node_send_output_bytes with parameters encoded from a dict."},
    {"send_buffer", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(py_send_buffer)),
     METH_FASTCALL, "dora_node_send_output_bytes of host bytes read in place (buffer protocol)."},
    {"send_array", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(py_send_array)),
     METH_FASTCALL, "dora_node_send_output with parameters encoded from a dict."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_dora_node",
                      "Per-send hot path of dora_amd.node (native, like the reference's PyO3 node).",
                      -1, methods, nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__dora_node(void) { return PyModule_Create(&module); }
