// median_slice_probe.hip — measurement tool (not product): the packed 16-bit
// lane-group median (128 < K <= 1024) with its selections side by side:
// byte-wise counting with v_sad_u8 (SEL 1), the radix select on bit planes
// (SEL 2), the same with the planes built group by group as the loads land
// (SEL 3), at 2 or 3 waves per SIMD, and the LDS-DMA streamed form
// (median_pk16_stream_kernel); timed and compared bit for bit by
// tools/median_slice_probe.py.
#include "../fedml_amd/csrc/median.hip"

extern "C" int fedagg_set_error_internal(int code, const char*) { return code; }

namespace {
template <int SEL, int WPE, class E>
int probe_sel(const uint16_t* const* src, int K, int64_t N, uint16_t* out, hipStream_t st) {
  if (K <= 256) return launch_median_pk16_lanes<2, 128, E, 256, SEL, WPE>(src, K, N, out, st);
  if (K <= 512) return launch_median_pk16_lanes<4, 128, E, 256, SEL, WPE>(src, K, N, out, st);
  if (K <= 1024) return launch_median_pk16_lanes<8, 128, E, 256, SEL, WPE>(src, K, N, out, st);
  return 1;
}
template <int R, class E>
int probe_stream(const uint16_t* const* src, int K, int64_t N, uint16_t* out, hipStream_t st) {
  if (K <= 256) return launch_median_pk16_stream<256 / R, R, E>(src, K, N, out, st);
  if (K <= 512) return launch_median_pk16_stream<512 / R, R, E>(src, K, N, out, st);
  if (K <= 1024) return launch_median_pk16_stream<1024 / R, R, E>(src, K, N, out, st);
  return 1;
}
template <class E>
int probe_variant(int v, const uint16_t* const* s, int K, int64_t N, uint16_t* o, hipStream_t st) {
  switch (v) {
    case 1: return probe_sel<1, 2, E>(s, K, N, o, st);
    case 2: return probe_sel<2, 2, E>(s, K, N, o, st);
    case 3: return probe_sel<3, 2, E>(s, K, N, o, st);
    case 4: return probe_sel<2, 3, E>(s, K, N, o, st);
    case 5: return probe_sel<3, 3, E>(s, K, N, o, st);
    case 6: return probe_stream<128, E>(s, K, N, o, st);
    case 7: return probe_stream<64, E>(s, K, N, o, st);
  }
  return 1;
}
}  // namespace

extern "C" const char* slice_probe_name(int v) {
  static const char* n[] = {"", "count_w2", "slice_w2", "slice_pipe_w2", "slice_w3", "slice_pipe_w3", "stream_r128", "stream_r64"};
  return (v >= 1 && v <= 7) ? n[v] : "";
}

// v: variant (slice_probe_name); f16: 0 bf16 rows, 1 f16 rows
extern "C" int slice_probe_launch(int v, int f16, const void* src, int K, int64_t N, void* out, void* stream) {
  auto s = static_cast<const uint16_t* const*>(src);
  auto o = static_cast<uint16_t*>(out);
  auto st = static_cast<hipStream_t>(stream);
  return f16 ? probe_variant<MedF16>(v, s, K, N, o, st) : probe_variant<MedBF16>(v, s, K, N, o, st);
}
