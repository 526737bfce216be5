// adam_probe.hip — measurement tool (not product): tile shapes (U clients x V
// packs per lane) of the reduction kernel of fedml_amd/csrc/fedagg.hip at
// config 5 (64 clients x 4,194,304 fp32) for the three fp32 epilogues: plain
// FedAvg store, fused server SGD(+momentum), fused server Adam.  Timed by
// tools/adam_probe.py.
#include "../fedml_amd/csrc/fedagg.hip"

namespace {
template <int U, int V>
int probe_launch(int epi_kind, const float* const* src, const float* w, int K, int64_t N, float* p, float* m,
                 float* v, const float* sc, int first, hipStream_t st) {
  constexpr int BS = 256;
  const int64_t grid = ((N + 3) / 4 + int64_t(BS) * V - 1) / (int64_t(BS) * V);
  Seg<OpF32> s{src, N};
  InlW<float> iw;
  inline_weights<float>(w, K, &iw);
  if (epi_kind == 0) {
    hipLaunchKernelGGL((reduce_kernel<OpF32, U, V, true, true, BS, StoreEpi<OpF32>, InlW<float>>), dim3(unsigned(grid)),
                       dim3(BS), 0, st, s, StoreEpi<OpF32>{p}, iw, K);
  } else if (epi_kind == 1) {
    SgdEpi epi{p, m, -1.0f, 0.9f, first};
    hipLaunchKernelGGL((reduce_kernel<OpF32, U, V, true, true, BS, SgdEpi, InlW<float>>), dim3(unsigned(grid)),
                       dim3(BS), 0, st, s, epi, iw, K);
  } else {
    AdamEpi epi{p, m, v, sc[0], sc[1], sc[2], sc[3], sc[4], sc[5], first};
    hipLaunchKernelGGL((reduce_fused_kernel<OpF32, U, V, true, true, BS, AdamEpi, InlW<float>>),
                       dim3(unsigned(grid)), dim3(BS), 0, st, s, epi, iw, K);
  }
  return hipGetLastError();
}
}  // namespace

extern "C" const char* adam_probe_name(int i) {
  static const char* n[] = {"U4V4", "U2V4", "U1V4", "U1V2", "U1V1", "U2V2", "U8V1"};
  return (i >= 0 && i < 7) ? n[i] : "";
}

// w and sc are HOST arrays (K <= 256 weights; the six Adam scalars)
extern "C" int adam_probe_launch(int i, int epi_kind, const void* src, const float* w, int K, int64_t N, void* p,
                                 void* m, void* v, const float* sc, int first, void* stream) {
  auto s = reinterpret_cast<const float* const*>(src);
  auto P = reinterpret_cast<float*>(p), M = reinterpret_cast<float*>(m), Vv = reinterpret_cast<float*>(v);
  auto st = reinterpret_cast<hipStream_t>(stream);
  if (K < 1 || K > 256 || N < 1 || (N & 3)) return -1;
  switch (i) {
    case 0: return probe_launch<4, 4>(epi_kind, s, w, K, N, P, M, Vv, sc, first, st);
    case 1: return probe_launch<2, 4>(epi_kind, s, w, K, N, P, M, Vv, sc, first, st);
    case 2: return probe_launch<1, 4>(epi_kind, s, w, K, N, P, M, Vv, sc, first, st);
    case 3: return probe_launch<1, 2>(epi_kind, s, w, K, N, P, M, Vv, sc, first, st);
    case 4: return probe_launch<1, 1>(epi_kind, s, w, K, N, P, M, Vv, sc, first, st);
    case 5: return probe_launch<2, 2>(epi_kind, s, w, K, N, P, M, Vv, sc, first, st);
    case 6: return probe_launch<8, 1>(epi_kind, s, w, K, N, P, M, Vv, sc, first, st);
    default: return -1;
  }
}
