// The pack kernels of the AQL path (aql.cpp): the same device code as the HIP-launched
// signalling packs (pack_device.h), as plain extern "C" entry points that take no hidden kernel
// arguments (grid size in the arguments, workgroup id from its SGPR), so that a node can
// dispatch them with raw AQL packets on its own HSA queue.  Built as a standalone gfx950 code
// object (dora_amd/build.py) and embedded in libdora_gpu.so.
#include "pack_device.h"

using dora::pack::AqlPackArgs;
using dora::pack::kThreads;

extern "C" __global__ __launch_bounds__(kThreads) void dora_aql_pack_u4(AqlPackArgs a) {
  dora::pack::pack_body<4, 2>(a, __builtin_amdgcn_workgroup_id_x(), a.grid);
}

extern "C" __global__ __launch_bounds__(kThreads) void dora_aql_pack_u8(AqlPackArgs a) {
  dora::pack::pack_body<8, 2>(a, __builtin_amdgcn_workgroup_id_x(), a.grid);
}
