// abi_test.cpp — drives libfedagg.so through include/fedagg.h alone (no
// Python, no torch): the C ABI is the drop-in boundary, so a C/C++ host (or a
// cgo / JNI shim) must be able to use it as is.  Device memory comes from the
// HIP runtime; every result is checked bit for bit against the C oracle
// (oracle/fedavg_oracle.c, linked in as test infrastructure).
//
//   built by tests/test_c_abi.py; run on an MI355X: ./abi_test  -> "ABI OK"
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/fedagg.h"

extern "C" {
void oracle_wsum_f32(const float* const* src, const float* w, int K, int64_t N, float* out);
void oracle_wsum_bf16(const uint16_t* const* src, const float* w, int K, int64_t N, uint16_t* out);
void oracle_wsum_i64_f32(const int64_t* const* src, const float* w, int K, int64_t N, float* out);
uint16_t oracle_f32_to_bf16(float f);
}

#define HIP_OK(x)                                                        \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      std::printf("HIP error %d at %s:%d\n", int(e_), __FILE__, __LINE__); \
      return 2;                                                          \
    }                                                                    \
  } while (0)

static uint64_t g_state = 88172645463325252ull;
static uint64_t next_u64() {  // xorshift64
  g_state ^= g_state << 13;
  g_state ^= g_state >> 7;
  g_state ^= g_state << 17;
  return g_state;
}
static float next_f32() { return float(int64_t(next_u64() % 2000001) - 1000000) * 1e-6f; }

template <class T>
static int upload_rows(const std::vector<std::vector<T>>& rows, std::vector<T*>& dev, T*** d_table) {
  const int K = int(rows.size());
  dev.resize(K);
  for (int i = 0; i < K; ++i) {
    HIP_OK(hipMalloc(&dev[i], rows[i].size() * sizeof(T) + 16));
    HIP_OK(hipMemcpy(dev[i], rows[i].data(), rows[i].size() * sizeof(T), hipMemcpyHostToDevice));
  }
  HIP_OK(hipMalloc(d_table, K * sizeof(T*)));
  HIP_OK(hipMemcpy(*d_table, dev.data(), K * sizeof(T*), hipMemcpyHostToDevice));
  return 0;
}

int main() {
  const int K = 7;
  const int64_t N = 1000003;  // ragged: the tail takes the scalar path
  // weights exactly as the reference: float32(double(n_i) / double(sum n))
  const int n[K] = {120, 7, 999, 455, 3, 61, 1000};
  double tot = 0;
  for (int i = 0; i < K; ++i) tot += n[i];
  std::vector<float> w(K);
  for (int i = 0; i < K; ++i) w[i] = float(double(n[i]) / tot);
  float* d_w;
  HIP_OK(hipMalloc(&d_w, K * sizeof(float)));
  HIP_OK(hipMemcpy(d_w, w.data(), K * sizeof(float), hipMemcpyHostToDevice));
  int failures = 0;

  // ---- fp32 FedAvg ---------------------------------------------------------
  {
    std::vector<std::vector<float>> rows(K, std::vector<float>(N));
    for (auto& r : rows)
      for (auto& x : r) x = next_f32();
    std::vector<float*> dev;
    float** d_src;
    if (upload_rows(rows, dev, &d_src)) return 2;
    float* d_out;
    HIP_OK(hipMalloc(&d_out, N * sizeof(float)));
    int rc = fedagg_wsum_f32(d_src, d_w, K, N, d_out, FEDAGG_ALIGNED16, nullptr);
    if (rc) {
      std::printf("fedagg_wsum_f32 rc=%d: %s\n", rc, fedagg_last_error());
      return 1;
    }
    // weights by value (FEDAGG_HOST_WEIGHTS): host array, same bits
    float* d_out2;
    HIP_OK(hipMalloc(&d_out2, N * sizeof(float)));
    rc = fedagg_wsum_f32(d_src, w.data(), K, N, d_out2, FEDAGG_ALIGNED16 | FEDAGG_HOST_WEIGHTS, nullptr);
    if (rc) {
      std::printf("host-weights rc=%d: %s\n", rc, fedagg_last_error());
      return 1;
    }
    HIP_OK(hipDeviceSynchronize());
    std::vector<float> got(N), got2(N), ref(N);
    HIP_OK(hipMemcpy(got.data(), d_out, N * sizeof(float), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(got2.data(), d_out2, N * sizeof(float), hipMemcpyDeviceToHost));
    std::vector<const float*> hp(K);
    for (int i = 0; i < K; ++i) hp[i] = rows[i].data();
    oracle_wsum_f32(hp.data(), w.data(), K, N, ref.data());
    if (std::memcmp(got.data(), ref.data(), N * 4) || std::memcmp(got2.data(), ref.data(), N * 4)) {
      std::printf("fp32 FedAvg differs from the oracle\n");
      ++failures;
    }
  }
  // ---- bf16 FedAvg (reference chain) ---------------------------------------
  {
    std::vector<std::vector<uint16_t>> rows(K, std::vector<uint16_t>(N));
    for (auto& r : rows)
      for (auto& x : r) x = oracle_f32_to_bf16(next_f32());
    std::vector<uint16_t*> dev;
    uint16_t** d_src;
    if (upload_rows(rows, dev, &d_src)) return 2;
    uint16_t* d_out;
    HIP_OK(hipMalloc(&d_out, N * 2));
    int rc = fedagg_wsum_bf16(d_src, d_w, K, N, d_out, FEDAGG_ACC_REFERENCE, FEDAGG_ALIGNED16, nullptr);
    if (rc) {
      std::printf("fedagg_wsum_bf16 rc=%d: %s\n", rc, fedagg_last_error());
      return 1;
    }
    HIP_OK(hipDeviceSynchronize());
    std::vector<uint16_t> got(N), ref(N);
    HIP_OK(hipMemcpy(got.data(), d_out, N * 2, hipMemcpyDeviceToHost));
    std::vector<const uint16_t*> hp(K);
    for (int i = 0; i < K; ++i) hp[i] = rows[i].data();
    oracle_wsum_bf16(hp.data(), w.data(), K, N, ref.data());
    if (std::memcmp(got.data(), ref.data(), N * 2)) {
      std::printf("bf16 FedAvg differs from the oracle\n");
      ++failures;
    }
  }
  // ---- int64 -> fp32 (BatchNorm counters) -----------------------------------
  {
    std::vector<std::vector<int64_t>> rows(K, std::vector<int64_t>(4099));
    for (auto& r : rows)
      for (auto& x : r) x = int64_t(next_u64() % (1ull << 41)) - (1ll << 40);
    std::vector<int64_t*> dev;
    int64_t** d_src;
    if (upload_rows(rows, dev, &d_src)) return 2;
    float* d_out;
    HIP_OK(hipMalloc(&d_out, 4099 * 4));
    int rc = fedagg_wsum_i64_f32(d_src, d_w, K, 4099, d_out, FEDAGG_ALIGNED16, nullptr);
    if (rc) {
      std::printf("fedagg_wsum_i64_f32 rc=%d: %s\n", rc, fedagg_last_error());
      return 1;
    }
    HIP_OK(hipDeviceSynchronize());
    std::vector<float> got(4099), ref(4099);
    HIP_OK(hipMemcpy(got.data(), d_out, 4099 * 4, hipMemcpyDeviceToHost));
    std::vector<const int64_t*> hp(K);
    for (int i = 0; i < K; ++i) hp[i] = rows[i].data();
    oracle_wsum_i64_f32(hp.data(), w.data(), K, 4099, ref.data());
    if (std::memcmp(got.data(), ref.data(), 4099 * 4)) {
      std::printf("int64 FedAvg differs from the oracle\n");
      ++failures;
    }
  }
  // ---- a small device round in one launch (fedagg_device_round_f32) ---------
  {
    // config 1's shape: 4 clients x {7840 weights, 10 biases} fp32, host
    // weights, every pointer in the kernel arguments
    const int KS = 4, T = 2;
    const int64_t numels[T] = {7840, 10};
    const int32_t codes[T] = {FEDAGG_DT_F32, FEDAGG_DT_F32};
    const float ws[KS] = {0.1f, 0.2f, 0.3f, 0.4f};
    std::vector<std::vector<float>> host(T * KS);
    std::vector<float*> dsrc(T * KS);
    for (int t = 0; t < T; ++t)
      for (int i = 0; i < KS; ++i) {
        auto& h = host[t * KS + i];
        h.resize(numels[t]);
        for (auto& x : h) x = next_f32();
        HIP_OK(hipMalloc(&dsrc[t * KS + i], numels[t] * 4));
        HIP_OK(hipMemcpy(dsrc[t * KS + i], h.data(), numels[t] * 4, hipMemcpyHostToDevice));
      }
    std::vector<float*> dout(T);
    for (int t = 0; t < T; ++t) HIP_OK(hipMalloc(&dout[t], numels[t] * 4));
    int rc = fedagg_device_round_f32(reinterpret_cast<const void* const*>(dsrc.data()), codes, numels, T, KS, ws,
                                     reinterpret_cast<void* const*>(dout.data()), nullptr);
    if (rc) {
      std::printf("fedagg_device_round_f32 rc=%d: %s\n", rc, fedagg_last_error());
      return 1;
    }
    HIP_OK(hipDeviceSynchronize());
    for (int t = 0; t < T; ++t) {
      std::vector<float> got(numels[t]), ref(numels[t]);
      HIP_OK(hipMemcpy(got.data(), dout[t], numels[t] * 4, hipMemcpyDeviceToHost));
      std::vector<const float*> hp(KS);
      for (int i = 0; i < KS; ++i) hp[i] = host[t * KS + i].data();
      oracle_wsum_f32(hp.data(), ws, KS, numels[t], ref.data());
      if (std::memcmp(got.data(), ref.data(), numels[t] * 4)) {
        std::printf("device round key %d differs from the oracle\n", t);
        ++failures;
      }
    }
    // ---- the same clients through a batched launch (fedagg_wsum_fedopt_batch):
    // FEDAGG_FEDOPT_AVG of key 0 into a parameter buffer equals the plain average
    float** d_tab;
    HIP_OK(hipMalloc(&d_tab, KS * sizeof(float*)));
    HIP_OK(hipMemcpy(d_tab, dsrc.data(), KS * sizeof(float*), hipMemcpyHostToDevice));
    float* d_param;
    HIP_OK(hipMalloc(&d_param, numels[0] * 4));
    int dev = 0;
    HIP_OK(hipGetDevice(&dev));
    fedagg_fedopt_launch l;
    std::memset(&l, 0, sizeof(l));
    l.d_src = d_tab;
    l.weights = ws;
    l.d_param = d_param;
    l.N = numels[0];
    l.K = KS;
    l.opt = FEDAGG_FEDOPT_AVG;
    l.device = dev;
    l.flags = FEDAGG_ALIGNED16 | FEDAGG_HOST_WEIGHTS;
    rc = fedagg_wsum_fedopt_batch(&l, 1);
    if (rc) {
      std::printf("fedagg_wsum_fedopt_batch rc=%d: %s\n", rc, fedagg_last_error());
      return 1;
    }
    HIP_OK(hipDeviceSynchronize());
    std::vector<float> a(numels[0]), b(numels[0]);
    HIP_OK(hipMemcpy(a.data(), d_param, numels[0] * 4, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(b.data(), dout[0], numels[0] * 4, hipMemcpyDeviceToHost));
    if (std::memcmp(a.data(), b.data(), numels[0] * 4)) {
      std::printf("batched FedAvg launch differs from the device round\n");
      ++failures;
    }
  }
  // ---- errors are reported, not crashed on ----------------------------------
  if (fedagg_wsum_f32(nullptr, d_w, 0, 10, nullptr, 0, nullptr) != FEDAGG_EINVAL ||
      std::strstr(fedagg_last_error(), "K must be") == nullptr) {
    std::printf("argument validation broken\n");
    ++failures;
  }
  if (failures) return 1;
  std::printf("ABI OK (fedagg_version %d)\n", fedagg_version());
  return 0;
}
