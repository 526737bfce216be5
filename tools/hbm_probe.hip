// hbm_probe.hip — measurement tool (not product): the achievable HBM rates on
// this MI355X for the access shapes the aggregation kernel uses, so the
// kernel's roofline fraction can be read against a measured ceiling as well
// as the 8 TB/s spec (cdna_hip_programming.md §5.4 rule 10).
//
//   probe_read   : every lane streams 16-byte non-temporal loads, U in flight,
//                  folds them into a register sum, writes one float per lane
//   probe_copy   : 16-byte nt load -> 16-byte nt store
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void probe_read(const f32x4* __restrict__ src, int64_t n4, float* __restrict__ out) {
  const int64_t stride = int64_t(gridDim.x) * 256;
  int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += x[u];
  }
  for (; i < n4; i += stride) acc += __builtin_nontemporal_load(src + i);
  out[int64_t(blockIdx.x) * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

__global__ __launch_bounds__(256) void probe_copy(const f32x4* __restrict__ src, f32x4* __restrict__ dst, int64_t n4) {
  const int64_t stride = int64_t(gridDim.x) * 256;
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n4; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

extern "C" int probe_read_launch(const void* src, int64_t n4, void* out, int grid, int unroll, void* stream) {
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto p = reinterpret_cast<const f32x4*>(src);
  auto o = reinterpret_cast<float*>(out);
  switch (unroll) {
    case 4: hipLaunchKernelGGL(probe_read<4>, dim3(grid), dim3(256), 0, s, p, n4, o); break;
    case 8: hipLaunchKernelGGL(probe_read<8>, dim3(grid), dim3(256), 0, s, p, n4, o); break;
    case 16: hipLaunchKernelGGL(probe_read<16>, dim3(grid), dim3(256), 0, s, p, n4, o); break;
    default: return -1;
  }
  return hipGetLastError();
}

extern "C" int probe_copy_launch(const void* src, void* dst, int64_t n4, int grid, void* stream) {
  hipLaunchKernelGGL(probe_copy, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const f32x4*>(src), reinterpret_cast<f32x4*>(dst), n4);
  return hipGetLastError();
}
