// median_probe.hip — measurement tool (not product): variants of the
// coordinate-wise median kernel of fedml_amd/csrc/fedagg.hip, timed by
// tools/median_probe.py on the GPU box to choose the shipped launch shape.
#include "../fedml_amd/csrc/fedagg.hip"

namespace {
template <int BS, bool PRIO>
int probe_launch(const float* const* src, int64_t N, float* out, hipStream_t st) {
  const int64_t grid = (N + BS - 1) / BS;
  hipLaunchKernelGGL((median_kernel<128, true, BS, PRIO>), dim3(unsigned(grid)), dim3(BS), 0, st, src, 128, N, out);
  return hipGetLastError();
}
}  // namespace

extern "C" const char* median_probe_name(int v) {
  static const char* names[] = {"bs256", "bs256_prio", "bs64", "bs64_prio", "bs128", "bs512"};
  return (v >= 0 && v < 6) ? names[v] : "";
}

// K is fixed at 128 (the full kernel); src is a device table of 128 row pointers
extern "C" int median_probe_launch(int v, const void* src, int64_t N, void* out, void* stream) {
  if (N <= 0 || N > (int64_t(1) << 30)) return -1;
  auto s = reinterpret_cast<const float* const*>(src);
  auto o = reinterpret_cast<float*>(out);
  auto st = reinterpret_cast<hipStream_t>(stream);
  switch (v) {
    case 0: return probe_launch<256, false>(s, N, o, st);
    case 1: return probe_launch<256, true>(s, N, o, st);
    case 2: return probe_launch<64, false>(s, N, o, st);
    case 3: return probe_launch<64, true>(s, N, o, st);
    case 4: return probe_launch<128, false>(s, N, o, st);
    case 5: return probe_launch<512, false>(s, N, o, st);
    default: return -1;
  }
}
