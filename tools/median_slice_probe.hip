// median_slice_probe.hip — measurement tool (not product): the packed 16-bit
// median above 128 clients (K <= 1024) as fedagg_median dispatches it (the
// LDS-DMA streamed bit-plane kernels, median.hip) beside the register form of
// the same selection (median_pk16_lanes_kernel<PLANES>) and the sorting
// networks (median_pk16_lanes_kernel, K > 1024 in the product) and the column
// kernel at 32 words per lane in 8-wave blocks (4 waves per SIMD), timed and
// compared bit for bit by tools/median_slice_probe.py.  The forms measured
// and dropped in round 6 (byte-wise counting, the per-wave and grid-stride
// streams, R = 64 pair tiles) are in NOTES.md §5b with their numbers.
#include "../fedml_amd/csrc/median.hip"

extern "C" int fedagg_set_error_internal(int code, const char*) { return code; }

namespace {
template <bool PLANES, class E>
int probe_lanes(const uint16_t* const* src, int K, int64_t N, uint16_t* out, hipStream_t st) {
  if (K <= 256) return launch_median_pk16_lanes<2, 128, E, 256, PLANES>(src, K, N, out, st);
  if (K <= 512) return launch_median_pk16_lanes<4, 128, E, 256, PLANES>(src, K, N, out, st);
  if (K <= 1024) return launch_median_pk16_lanes<8, 128, E, 256, PLANES>(src, K, N, out, st);
  return 1;
}
template <class E>
int probe_col32(const uint16_t* const* src, int K, int64_t N, uint16_t* out, hipStream_t st) {
  if (K <= 256) return launch_median_pk16_colstream<4, 32, 8, E>(src, K, N, out, st);
  if (K <= 512) return launch_median_pk16_colstream<8, 32, 8, E>(src, K, N, out, st);
  return median_dispatch<E>(src, K, N, out, true, st);
}
// K <= 128: one lane per column pair holding all 128 clients, bit planes
template <class E>
int probe_k128_planes(const uint16_t* const* src, int K, int64_t N, uint16_t* out, hipStream_t st) {
  if (K <= 128) return launch_median_pk16_lanes<1, 128, E, 256, true>(src, K, N, out, st);
  return median_dispatch<E>(src, K, N, out, true, st);
}
template <class E>
int probe_small_planes(const uint16_t* const* src, int K, int64_t N, uint16_t* out, hipStream_t st) {
  if (K <= 32) return launch_median_pk16_lanes<1, 32, E, 256, true>(src, K, N, out, st);
  if (K <= 64) return launch_median_pk16_lanes<1, 64, E, 256, true>(src, K, N, out, st);
  if (K <= 128) return launch_median_pk16_lanes<1, 128, E, 256, true>(src, K, N, out, st);
  return median_dispatch<E>(src, K, N, out, true, st);
}
// 513..1024 clients through the column kernel (8 lanes per column, 8-wave blocks, one per CU)
template <class E>
int probe_col1024(const uint16_t* const* src, int K, int64_t N, uint16_t* out, hipStream_t st) {
  if (K > 512 && K <= 1024) return launch_median_pk16_colstream<8, 64, 8, E>(src, K, N, out, st);
  return median_dispatch<E>(src, K, N, out, true, st);
}
template <class E>
int probe_variant(int v, const uint16_t* const* s, int K, int64_t N, uint16_t* o, hipStream_t st) {
  switch (v) {
    case 1: return median_dispatch<E>(s, K, N, o, true, st);
    case 2: return probe_lanes<true, E>(s, K, N, o, st);
    case 3: return probe_lanes<false, E>(s, K, N, o, st);
    case 4: return probe_col32<E>(s, K, N, o, st);
    case 5: return probe_k128_planes<E>(s, K, N, o, st);
    case 6: return probe_small_planes<E>(s, K, N, o, st);
    case 7: return probe_col1024<E>(s, K, N, o, st);
  }
  return 1;
}
}  // namespace

extern "C" const char* slice_probe_name(int v) {
  static const char* n[] = {"", "shipped", "planes_regs", "networks_regs", "col_r32_w8", "k128_planes",
                           "small_planes", "col_k1024"};
  return (v >= 1 && v <= 7) ? n[v] : "";
}

// v: variant (slice_probe_name); f16: 0 bf16 rows, 1 f16 rows
extern "C" int slice_probe_launch(int v, int f16, const void* src, int K, int64_t N, void* out, void* stream) {
  auto s = static_cast<const uint16_t* const*>(src);
  auto o = static_cast<uint16_t*>(out);
  auto st = static_cast<hipStream_t>(stream);
  return f16 ? probe_variant<MedF16>(v, s, K, N, o, st) : probe_variant<MedBF16>(v, s, K, N, o, st);
}
