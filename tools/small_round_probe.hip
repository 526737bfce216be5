// small_round_probe.hip — measurement tool (not product): the host-side floor
// of one small FedAvg round (config 1: 4 clients x 7,850 fp32; config 2: 32 x
// 62,006) done as ONE native sequence, to choose the shape of the small-round
// path of fedml_amd.agg_operator.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/_build/small_round_probe tools/small_round_probe.hip
//   tools/_build/small_round_probe            # prints one JSON line per variant
//
// Variants (median of 2000 rounds after 200 warm-up, wall clock on the host):
//   empty     : an empty kernel launch + hipStreamSynchronize (launch/complete floor)
//   copy      : pack (memcpy) into pinned -> hipMemcpyAsync H2D -> reduce kernel ->
//               hipMemcpyAsync D2H -> sync -> unpack (memcpy)
//   zerocopy  : pack into pinned -> reduce kernel reading the pinned staging and
//               writing the pinned result directly over PCIe -> sync -> unpack
//   cpu       : the same weighted sum on the host, one thread (reference scale)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void empty_kernel() {}

// rows: [K][L] fp32; one thread per element, clients in order, two roundings
__global__ void wsum_kernel(const float* __restrict__ rows, const float* __restrict__ w, int K, int L,
                            float* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= L) return;
  float acc = rows[e] * w[0];
  for (int i = 1; i < K; ++i) acc = acc + rows[int64_t(i) * L + e] * w[i];
  out[e] = acc;
}

struct WArg {
  float w[64];
};
__global__ void wsum_kernel_inl(const float* __restrict__ rows, WArg wa, int K, int L, float* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= L) return;
  float acc = rows[e] * wa.w[0];
  for (int i = 1; i < K; ++i) acc = acc + rows[int64_t(i) * L + e] * wa.w[i];
  out[e] = acc;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int run(int K, int L, const char* cfg) {
  const int reps = 2000, warm = 200;
  std::vector<std::vector<float>> clients(K, std::vector<float>(L));
  for (int i = 0; i < K; ++i)
    for (int e = 0; e < L; ++e) clients[i][e] = float((e * 7 + i * 13) % 101) * 0.01f;
  std::vector<float> result(L);
  WArg wa{};
  for (int i = 0; i < K; ++i) wa.w[i] = 1.0f / K;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  float *stage = nullptr, *res_h = nullptr, *rows_d = nullptr, *out_d = nullptr, *w_d = nullptr;
  CK(hipHostMalloc(&stage, size_t(K) * L * 4, hipHostMallocDefault));
  CK(hipHostMalloc(&res_h, size_t(L) * 4, hipHostMallocDefault));
  CK(hipMalloc(&rows_d, size_t(K) * L * 4));
  CK(hipMalloc(&out_d, size_t(L) * 4));
  CK(hipMalloc(&w_d, 64 * 4));
  float *stage_c = nullptr, *res_c = nullptr;  // coherent, device-mapped
  CK(hipHostMalloc(&stage_c, size_t(K) * L * 4, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc(&res_c, size_t(L) * 4, hipHostMallocCoherent | hipHostMallocMapped));
  float *stage_cd = nullptr, *res_cd = nullptr;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&stage_cd), stage_c, 0));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&res_cd), res_c, 0));
  const dim3 blk(256), grd((L + 255) / 256);
  std::vector<double> t;

  // empty
  t.clear();
  for (int r = 0; r < reps + warm; ++r) {
    const double a = now_us();
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st);
    CK(hipStreamSynchronize(st));
    if (r >= warm) t.push_back(now_us() - a);
  }
  printf("{\"cfg\": \"%s\", \"variant\": \"empty\", \"us\": %.2f}\n", cfg, median(t));

  // copy
  t.clear();
  for (int r = 0; r < reps + warm; ++r) {
    const double a = now_us();
    for (int i = 0; i < K; ++i) memcpy(stage + size_t(i) * L, clients[i].data(), size_t(L) * 4);
    CK(hipMemcpyAsync(rows_d, stage, size_t(K) * L * 4, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(wsum_kernel_inl, grd, blk, 0, st, rows_d, wa, K, L, out_d);
    CK(hipMemcpyAsync(res_h, out_d, size_t(L) * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    memcpy(result.data(), res_h, size_t(L) * 4);
    if (r >= warm) t.push_back(now_us() - a);
  }
  printf("{\"cfg\": \"%s\", \"variant\": \"copy\", \"us\": %.2f, \"check\": %.6f}\n", cfg, median(t), result[L / 2]);

  // zerocopy
  t.clear();
  for (int r = 0; r < reps + warm; ++r) {
    const double a = now_us();
    for (int i = 0; i < K; ++i) memcpy(stage_c + size_t(i) * L, clients[i].data(), size_t(L) * 4);
    hipLaunchKernelGGL(wsum_kernel_inl, grd, blk, 0, st, stage_cd, wa, K, L, res_cd);
    CK(hipStreamSynchronize(st));
    memcpy(result.data(), res_c, size_t(L) * 4);
    if (r >= warm) t.push_back(now_us() - a);
  }
  printf("{\"cfg\": \"%s\", \"variant\": \"zerocopy\", \"us\": %.2f, \"check\": %.6f}\n", cfg, median(t),
         result[L / 2]);

  // cpu
  t.clear();
  for (int r = 0; r < reps + warm; ++r) {
    const double a = now_us();
    for (int e = 0; e < L; ++e) result[e] = clients[0][e] * wa.w[0];
    for (int i = 1; i < K; ++i)
      for (int e = 0; e < L; ++e) result[e] = result[e] + clients[i][e] * wa.w[i];
    if (r >= warm) t.push_back(now_us() - a);
  }
  printf("{\"cfg\": \"%s\", \"variant\": \"cpu1\", \"us\": %.2f, \"check\": %.6f}\n", cfg, median(t), result[L / 2]);
  return 0;
}

int main() {
  if (run(4, 7850, "cfg1")) return 1;
  if (run(32, 62006, "cfg2")) return 1;
  return 0;
}
