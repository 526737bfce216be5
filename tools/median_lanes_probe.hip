// median_lanes_probe.hip — measurement tool (not product): launch shapes of
// the lane-group median kernel of fedml_amd/csrc/fedagg.hip for 128 < K <= 1024
// (P lanes per column x R values per lane), timed by
// tools/median_lanes_probe.py.  (profiles/r02/median_lanes_probe.json also
// holds "ff" rows: a fused last level -- a plain min against the partner's
// mirrored register, then max3 -- measured once and not kept: -4 % to +6 %.)
#include "../fedml_amd/csrc/fedagg.hip"

namespace {
template <int P, int R, int BS = 256>
int probe_lanes(const float* const* src, int K, int64_t N, float* out, hipStream_t st) {
  if (K > P * R) return 1;
  const int64_t grid = (N * P + BS - 1) / BS;
  if (K == P * R)
    hipLaunchKernelGGL((median_lanes_kernel<P, R, true, MedF32, BS>), dim3(unsigned(grid)), dim3(BS), 0, st, src,
                       K, N, out);
  else
    hipLaunchKernelGGL((median_lanes_kernel<P, R, false, MedF32, BS>), dim3(unsigned(grid)), dim3(BS), 0, st, src,
                       K, N, out);
  return hipGetLastError();
}
}  // namespace

extern "C" const char* lanes_probe_name(int i) {
  static const char* n[] = {"4x64", "8x64", "4x128", "8x128", "2x128", "4x128bs64", "4x128bs128", "8x128bs64"};
  return (i >= 0 && i < 8) ? n[i] : "";
}

extern "C" int lanes_probe_launch(int i, const void* src, int K, int64_t N, void* out, void* stream) {
  auto s = static_cast<const float* const*>(src);
  auto o = static_cast<float*>(out);
  auto st = static_cast<hipStream_t>(stream);
  switch (i) {
    case 0: return probe_lanes<4, 64>(s, K, N, o, st);
    case 1: return probe_lanes<8, 64>(s, K, N, o, st);
    case 2: return probe_lanes<4, 128>(s, K, N, o, st);
    case 3: return probe_lanes<8, 128>(s, K, N, o, st);
    case 4: return probe_lanes<2, 128>(s, K, N, o, st);
    case 5: return probe_lanes<4, 128, 64>(s, K, N, o, st);
    case 6: return probe_lanes<4, 128, 128>(s, K, N, o, st);
    case 7: return probe_lanes<8, 128, 64>(s, K, N, o, st);
  }
  return 1;
}
