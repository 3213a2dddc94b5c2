"""ctypes binding of libdora_gpu.so (include/dora_gpu.h) and of the test hooks in
libdora_gpu_testing.so (include/dora_gpu_testing.h).

The library is built in-tree (dora_amd/lib/, `python -m dora_amd.build`).  There is no CPU
fallback: if the library is missing, importing the data plane raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_size_t,
                    c_uint8, c_uint32, c_uint64, c_void_p)

from .arrow_c import ArrowArray, ArrowSchema

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.path.join(LIB_DIR, "libdora_gpu.so")
TESTING_PATH = os.path.join(LIB_DIR, "libdora_gpu_testing.so")

ARROW_DEVICE_CPU = 1
ARROW_DEVICE_ROCM = 10
ARROW_DEVICE_ROCM_HOST = 11

DORA_OK = 0
ERRORS = {-1: "invalid", -2: "hip", -3: "too_small", -4: "unsupported", -5: "closed",
          -6: "timeout", -7: "not_found"}


class DoraGpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{ERRORS.get(code, code)}] {msg}")
        self.code = code


class UnsupportedType(DoraGpuError):
    pass


class VecU8(ctypes.Structure):
    """Vec_uint8_t of include/dora_operator_api.h."""
    _fields_ = [("ptr", c_void_p), ("len", c_size_t), ("cap", c_size_t)]


class DoraResult(ctypes.Structure):
    """DoraResult_t of include/dora_operator_api.h (error NULL: success)."""
    _fields_ = [("error", POINTER(VecU8))]


# name -> (restype, argtypes); `int` restype means a status code that is checked.
_SIGS = {
    "dora_gpu_last_error": (c_char_p, []),
    "dora_gpu_version": (c_char_p, []),
    "dora_gpu_busy_stats": (c_int, [POINTER(c_uint64), POINTER(c_uint64)]),
    "dora_gpu_aql_dispatch_counts": (c_int, [c_int, POINTER(c_uint64), c_size_t, POINTER(c_size_t)]),
    "dora_gpu_aql_kernel_name": (c_char_p, [c_size_t]),
    "dora_gpu_aql_batch_stats": (c_int, [c_int, POINTER(c_uint64), POINTER(c_uint64),
                                         POINTER(c_uint64)]),
    "dora_gpu_aql_cp_signalled": (c_int, [c_int, POINTER(c_uint64)]),
    "dora_gpu_set_keep_awake": (c_int, [ctypes.c_double]),
    "dora_gpu_device_count": (c_int, [POINTER(c_int)]),
    "dora_gpu_set_device": (c_int, [c_int]),
    "dora_gpu_get_device": (c_int, [POINTER(c_int)]),
    "dora_gpu_stream_create": (c_int, [POINTER(c_void_p)]),
    "dora_gpu_stream_destroy": (c_int, [c_void_p]),
    "dora_gpu_stream_sync": (c_int, [c_void_p]),
    "dora_gpu_device_sync": (c_int, []),
    "dora_gpu_malloc": (c_int, [POINTER(c_void_p), c_size_t]),
    "dora_gpu_free": (c_int, [c_void_p]),
    "dora_gpu_host_alloc": (c_int, [POINTER(c_void_p), c_size_t]),
    "dora_gpu_host_free": (c_int, [c_void_p]),
    "dora_gpu_memcpy_async": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "dora_gpu_memset_async": (c_int, [c_void_p, c_int, c_size_t, c_void_p]),
    "dora_gpu_event_create": (c_int, [POINTER(c_void_p)]),
    "dora_gpu_event_destroy": (c_int, [c_void_p]),
    "dora_gpu_event_record": (c_int, [c_void_p, c_void_p]),
    "dora_gpu_event_sync": (c_int, [c_void_p]),
    "dora_gpu_event_elapsed_ms": (c_int, [c_void_p, c_void_p, POINTER(c_float)]),
    "dora_gpu_plan": (c_int, [POINTER(ArrowArray), POINTER(ArrowSchema), c_int32,
                              POINTER(c_void_p)]),
    "dora_gpu_plan_bytes": (c_int, [c_void_p, c_size_t, c_int32, POINTER(c_void_p)]),
    "dora_gpu_plan_compact": (c_int, [POINTER(ArrowArray), POINTER(ArrowSchema), c_int32,
                                      POINTER(c_void_p)]),
    "dora_node_set_compact": (c_int, [c_void_p, c_int]),
    "dora_gpu_plan_free": (None, [c_void_p]),
    "dora_gpu_plan_size": (c_size_t, [c_void_p]),
    "dora_gpu_plan_num_segments": (c_size_t, [c_void_p]),
    "dora_gpu_plan_segment": (c_int, [c_void_p, c_size_t, POINTER(c_void_p), POINTER(c_uint64),
                                      POINTER(c_uint64)]),
    "dora_gpu_plan_type_info": (c_int, [c_void_p, POINTER(c_uint8), c_size_t,
                                        POINTER(c_size_t)]),
    "dora_gpu_pack": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "dora_gpu_array_upload": (c_int, [POINTER(ArrowArray), POINTER(ArrowSchema),
                                      POINTER(ArrowArray)]),
    "dora_gpu_array_download": (c_int, [POINTER(ArrowArray), POINTER(ArrowSchema),
                                        POINTER(ArrowArray)]),
    "dora_gpu_sample_import": (c_int, [c_void_p, c_size_t, POINTER(c_uint8), c_size_t,
                                       POINTER(ArrowArray), POINTER(ArrowSchema)]),
    "dora_gpu_type_info_schema": (c_int, [POINTER(c_uint8), c_size_t, POINTER(ArrowSchema)]),
    "dora_gpu_array_release": (None, [POINTER(ArrowArray)]),
    "dora_gpu_schema_release": (None, [POINTER(ArrowSchema)]),
    "dora_gpu_csum64": (c_int, [c_void_p, c_size_t, c_void_p, c_void_p]),
    "dora_gpu_csum64_sync": (c_int, [c_void_p, c_size_t, c_void_p, POINTER(c_uint64)]),
    "dora_gpu_fill_splitmix": (c_int, [c_void_p, c_size_t, c_uint64, c_void_p]),
    # node API
    "dora_node_init": (c_int, [c_char_p, c_char_p, c_int, POINTER(c_void_p)]),
    "dora_node_init_from_env": (c_int, [POINTER(c_void_p)]),
    "dora_node_free": (None, [c_void_p]),
    "dora_node_stream": (c_void_p, [c_void_p]),
    "dora_node_dataflow_id": (c_char_p, [c_void_p]),
    "dora_node_id": (c_char_p, [c_void_p]),
    "dora_node_allocate_data_sample": (c_int, [c_void_p, c_size_t, POINTER(c_void_p)]),
    "dora_sample_data": (c_void_p, [c_void_p]),
    "dora_sample_len": (c_size_t, [c_void_p]),
    "dora_sample_discard": (None, [c_void_p, c_void_p]),
    # parameter / type-info byte strings go in as c_char_p (bytes objects, no copy)
    "dora_node_send_output_sample": (c_int, [c_void_p, c_char_p, c_char_p, c_size_t,
                                             c_char_p, c_size_t, c_void_p]),
    "dora_node_send_output": (c_int, [c_void_p, c_char_p, POINTER(ArrowArray),
                                      POINTER(ArrowSchema), c_int32, c_char_p, c_size_t]),
    "dora_node_send_output_bytes": (c_int, [c_void_p, c_char_p, c_void_p, c_size_t, c_int32,
                                            c_char_p, c_size_t]),
    "dora_node_send_output_ex": (c_int, [c_void_p, c_char_p, POINTER(ArrowArray),
                                         POINTER(ArrowSchema), c_int32, c_char_p, c_size_t,
                                         ctypes.c_uint32]),
    "dora_node_send_output_bytes_ex": (c_int, [c_void_p, c_char_p, c_void_p, c_size_t, c_int32,
                                               c_char_p, c_size_t, ctypes.c_uint32]),
    "dora_node_set_async_sends": (c_int, [c_void_p, c_int]),
    "dora_node_set_event_thread": (c_int, [c_void_p, c_int]),
    "dora_node_close_outputs": (c_int, [c_void_p, POINTER(c_char_p), c_size_t]),
    "dora_node_next_event": (c_int, [c_void_p, c_int64, POINTER(c_void_p)]),
    "dora_event_type": (c_int, [c_void_p]),
    "dora_event_id": (c_char_p, [c_void_p]),
    "dora_event_error": (c_char_p, [c_void_p]),
    "dora_event_data": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_size_t)]),
    "dora_event_is_device": (c_int, [c_void_p]),
    "dora_event_type_info": (c_int, [c_void_p, POINTER(POINTER(c_uint8)), POINTER(c_size_t)]),
    "dora_event_parameters": (c_int, [c_void_p, POINTER(POINTER(c_uint8)), POINTER(c_size_t)]),
    "dora_event_timestamp_ns": (c_uint64, [c_void_p]),
    "dora_event_array": (c_int, [c_void_p, POINTER(ArrowArray), POINTER(ArrowSchema)]),
    "dora_event_free": (None, [c_void_p]),
    "dora_node_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64),
                                POINTER(c_uint64)]),
    "dora_node_set_profiling": (c_int, [c_void_p, c_int]),
    "dora_node_set_timing_period": (c_int, [c_void_p, c_uint64]),
    "dora_node_fill_paths": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    "dora_node_host_bound_outputs": (c_int, [c_void_p, c_char_p, c_uint64, POINTER(c_uint64)]),
    "dora_node_host_paths": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64),
                                     POINTER(c_uint64), POINTER(c_uint64)]),
    "dora_node_plan_cache_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    "dora_node_dataflow_counters": (c_int, [c_void_p, c_char_p, POINTER(c_uint64),
                                            POINTER(c_uint64), POINTER(c_uint64)]),
    "dora_node_region_begin": (c_int, [c_void_p]),
    "dora_node_region_mark": (c_int, [c_void_p]),
    "dora_node_sync": (c_int, [c_void_p]),
    "dora_node_region_end": (c_int, [c_void_p, POINTER(c_double), POINTER(c_uint64),
                                     POINTER(c_uint64)]),
    "dora_node_pack_intervals": (c_int, [c_void_p, POINTER(c_double), c_size_t,
                                         POINTER(c_size_t)]),
    "dora_node_peer_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    "dora_node_bcast_ranks": (c_int, [c_void_p, POINTER(c_uint64)]),
    "dora_node_bcast_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64),
                                      POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64),
                                      POINTER(c_char_p)]),
    "dora_node_forward": (c_int, [c_void_p, c_char_p, c_void_p, c_char_p, c_size_t]),
    "dora_node_forward_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    "dora_node_send_profile": (c_int, [c_void_p, POINTER(c_double), c_size_t, POINTER(c_uint64)]),
    "dora_node_pack_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_double),
                                     POINTER(c_uint64)]),
    # shared-library operator helpers (include/dora_operator_api.h; used by operators)
    "dora_read_input_id": (c_void_p, [c_void_p]),
    "dora_free_input_id": (None, [c_void_p]),
    "dora_read_data": (VecU8, [c_void_p]),
    "dora_free_data": (None, [VecU8]),
    "dora_send_operator_output": (DoraResult, [c_void_p, c_char_p, c_void_p, c_size_t]),
    "dora_input_arrow": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_void_p)]),
    "dora_send_operator_output_arrow": (DoraResult, [c_void_p, c_char_p, c_void_p, c_void_p]),
    "dora_operator_error": (DoraResult, [c_char_p]),
    # daemon
    "dora_daemon_create": (c_int, [c_char_p, c_char_p, c_size_t, POINTER(c_void_p)]),
    "dora_daemon_run": (c_int, [c_void_p, c_int64]),
    "dora_daemon_request_stop": (c_int, [c_void_p]),
    "dora_daemon_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    "dora_daemon_listen_port": (c_int, [c_void_p, POINTER(c_int)]),
    "dora_daemon_remote_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64),
                                         POINTER(c_uint64)]),
    "dora_daemon_free": (None, [c_void_p]),
}

# libdora_gpu_testing.so (include/dora_gpu_testing.h): test and microbenchmark hooks, a library
# of their own so that the product ABI carries none of them
_TEST_SIGS = {
    "dora_gpu_test_fill_reached": (c_int, [c_void_p, c_uint64]),
    "dora_gpu_test_cp_arm": (c_int, [c_void_p, c_uint64]),
    "dora_gpu_test_l2_touch": (c_int, [c_void_p, c_size_t, c_void_p]),
    "dora_gpu_test_bar_alloc": (c_int, [c_int, c_size_t, POINTER(c_void_p)]),
    "dora_gpu_test_bar_write": (c_int, [c_int, c_void_p, c_void_p, c_size_t]),
    "dora_gpu_test_bar_free": (None, [c_void_p]),
    "dora_gpu_test_aql_hold": (c_int, [c_int, c_int]),
    "dora_gpu_test_reduce_timeout": (c_int, [c_uint64]),
    "dora_gpu_test_d2h_copy_probe": (c_int, [c_int, c_int, c_uint64, c_uint32, c_uint64, c_void_p]),
    "dora_gpu_test_stream_order_probe": (c_int, [c_int, c_int, c_uint64, c_uint32, c_void_p]),
    "dora_gpu_test_abandoned_slots": (c_int, [c_int, POINTER(c_uint32)]),
    "dora_gpu_test_keep_awake_stats": (c_int, [c_int, POINTER(c_uint64), POINTER(c_int)]),
    "dora_gpu_test_aql_ring_wc": (c_int, [c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "dora_gpu_test_bcast_group": (c_int, [c_int, c_void_p, c_uint64, POINTER(c_int),
                                          POINTER(c_int)]),
    "dora_gpu_test_l1_stale": (c_int, [c_int, c_int, POINTER(c_uint32), POINTER(c_uint32),
                                       POINTER(c_uint32)]),
    "dora_gpu_test_ide_output": (c_int, [c_char_p, c_char_p, c_char_p, c_void_p, c_size_t,
                                         c_void_p, c_size_t, c_uint64, c_uint64, c_void_p,
                                         c_void_p, c_size_t, c_int, c_void_p, c_size_t,
                                         POINTER(c_size_t)]),
    "dora_gpu_test_ide_inputs_closed": (c_int, [c_char_p, POINTER(c_char_p), POINTER(c_char_p),
                                                c_size_t, c_uint64, c_void_p, c_void_p,
                                                c_size_t, POINTER(c_size_t)]),
    "dora_gpu_test_ide_decode": (c_int, [c_void_p, c_size_t, c_char_p, c_size_t,
                                         POINTER(c_size_t)]),
    "dora_gpu_test_batch_args": (c_int, [c_size_t, POINTER(c_size_t), POINTER(c_uint64),
                                         POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64),
                                         POINTER(c_uint64), c_void_p, c_size_t,
                                         POINTER(ctypes.c_uint32)]),
}

_lib = None
_testing = None


def load(path: str = LIB_PATH):
    """Load libdora_gpu.so and declare every signature; raise if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `python -m dora_amd.build` (there is no CPU "
            "fallback for the device data plane)")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def load_testing():
    """Load libdora_gpu_testing.so (after the product library it links against) and declare
    the test hooks; raise if it is absent."""
    global _testing
    if _testing is not None:
        return _testing
    load()
    if not os.path.exists(TESTING_PATH):
        raise ImportError(f"{TESTING_PATH} is missing: build it with `python -m dora_amd.build`")
    lib = ctypes.CDLL(TESTING_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _TEST_SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _testing = lib
    return lib


def declared_symbols():
    return list(_SIGS)


def declared_test_symbols():
    return list(_TEST_SIGS)


def check(rc: int) -> int:
    if rc != DORA_OK:
        msg = _lib.dora_gpu_last_error().decode(errors="replace")
        cls = UnsupportedType if rc == -4 else DoraGpuError
        raise cls(rc, msg)
    return rc


def call(name: str, *args):
    lib = load_testing() if name.startswith("dora_gpu_test_") else load()
    return check(getattr(lib, name)(*args))
