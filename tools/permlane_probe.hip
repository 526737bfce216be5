// Probe (tool only): what __builtin_amdgcn_permlane16_swap returns on gfx950,
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/_build/permlane_probe tools/permlane_probe.hip
// for one wave whose lane i holds i in both operands.  Prints, per lane, the
// two results, so the xor-16 exchange can be built from them.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int* out) {
  const int x = threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(x, x + 1000, false, false);
  out[2 * threadIdx.x] = r[0];
  out[2 * threadIdx.x + 1] = r[1];
}

int main() {
  int* d;
  hipMalloc(&d, 128 * sizeof(int));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  int h[128];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int i = 0; i < 64; ++i) printf("%d:%d,%d%s", i, h[2 * i], h[2 * i + 1], (i % 8 == 7) ? "\n" : " ");
  hipFree(d);
  return 0;
}
