// median_probe.hip — measurement tool (not product): variants of the
// coordinate-wise median kernel of fedml_amd/csrc/fedagg.hip, timed by
// tools/median_probe.py on the GPU box to choose the shipped launch shape.
#include "../fedml_amd/csrc/fedagg.hip"

namespace {
// The first K > 128 kernel (shipped before the lane-group register sort,
// kept here as the A/B baseline).  The column no longer fits in one lane's
// registers.
// A workgroup stages a tile of kRadixCols consecutive columns x K clients in
// LDS (coalesced row segments in, stored column-major as order-preserving
// uint32 keys), then each wave selects one column's lower median with an
// 8-bit radix select over those keys: 4 passes of a 256-bin LDS histogram
// (ds_add), a wave prefix sum over the bins, and the digit that holds rank
// (K-1)/2.  Exact for every input: the key order is the float order with
// -0 < +0 (a ±0 tie at the median may return the other zero than torch's
// nth_element, as for the register kernel), and a column holding a NaN
// returns its first NaN in client order (the row index is found with an LDS
// atomic min while the tile is loaded).
constexpr int kRadixCols = 32;

// f32_order_key / f32_from_order_key: fedagg.hip (the radix-stream kernel)

// Column stride in LDS: >= KCAP and = 9 (mod 64), so the column-major writes
// of 64 consecutive columns hit 64 different banks and the 8 columns a wave
// instruction can touch start 9 banks apart.
template <int KCAP>
constexpr int radix_stride() {
  return KCAP + ((9 - KCAP % 64) + 64) % 64;
}

template <int KCAP>
__global__ __launch_bounds__(256) void median_radix_kernel(const float* const* __restrict__ src, int K, int64_t N,
                                                           float* __restrict__ out) {
  constexpr int C = kRadixCols, S = radix_stride<KCAP>();
  __shared__ uint32_t keys[C * S];
  __shared__ uint32_t hist[4][256];
  __shared__ int nan_row[C];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t col0 = int64_t(blockIdx.x) * C;
  const int ncols = int(min<int64_t>(C, N - col0));
  if (t < C) nan_row[t] = K;
  __syncthreads();

  // ---- tile load: thread t reads column t % C of rows t / C, t / C + 8, ...
  {
    const int cc = t % C;
    constexpr int RSTEP = 256 / C;
    if (cc < ncols) {
      int first_nan = K;
      int r = t / C;
      for (; r + 3 * RSTEP < K; r += 4 * RSTEP) {  // 4 rows in flight per thread
        float x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = __builtin_nontemporal_load(as_global(src[r + u * RSTEP]) + col0 + cc);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          keys[cc * S + r + u * RSTEP] = f32_order_key(__float_as_uint(x[u]));
          if (__builtin_isnan(x[u]) && first_nan == K) first_nan = r + u * RSTEP;
        }
      }
      for (; r < K; r += RSTEP) {
        const float x = __builtin_nontemporal_load(as_global(src[r]) + col0 + cc);
        keys[cc * S + r] = f32_order_key(__float_as_uint(x));
        if (__builtin_isnan(x) && first_nan == K) first_nan = r;
      }
      if (first_nan < K) atomicMin(&nan_row[cc], first_nan);
    }
  }
  __syncthreads();

  // ---- per-column radix select, one wave per column
  for (int c = w; c < ncols; c += 4) {
    const uint32_t* col = keys + c * S;
    uint32_t prefix = 0, pmask = 0;
    int rank = (K - 1) / 2;
#pragma unroll 1
    for (int shift = 24; shift >= 0; shift -= 8) {
#pragma unroll
      for (int b = lane; b < 256; b += 64) hist[w][b] = 0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int i = lane; i < K; i += 64) {
        const uint32_t k = col[i];
        if ((k & pmask) == prefix) atomicAdd(&hist[w][(k >> shift) & 0xffu], 1u);
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // lane owns bins 4*lane .. 4*lane+3; inclusive prefix sum over the wave
      uint32_t h[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) h[j] = hist[w][4 * lane + j];
      const int own = int(h[0] + h[1] + h[2] + h[3]);
      int incl = own;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      const int excl = incl - own;
      const uint64_t bal = __ballot(excl <= rank && rank < incl);
      const int L = __builtin_ctzll(bal);  // exactly one lane's bins hold the rank
      int digit = 4 * lane, below = excl;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (digit == 4 * lane + j && below + int(h[j]) <= rank) {
          below += int(h[j]);
          ++digit;
        }
      }
      digit = __builtin_amdgcn_readlane(digit, L);
      below = __builtin_amdgcn_readlane(below, L);
      prefix |= uint32_t(digit) << shift;
      pmask |= 0xffu << shift;
      rank -= below;
      __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) {
      const int nr = nan_row[c];
      out[col0 + c] = __uint_as_float(f32_from_order_key(nr < K ? col[nr] : prefix));
    }
  }
}

template <int KCAP>
int launch_median_radix(const float* const* src, int K, int64_t N, float* out, hipStream_t st) {
  const int64_t grid = (N + kRadixCols - 1) / kRadixCols;
  if (grid > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, "fedagg_median_f32: N too large");
  hipLaunchKernelGGL((median_radix_kernel<KCAP>), dim3(unsigned(grid)), dim3(256), 0, st, src, K, N, out);
  return check_launch("fedagg_median_f32");
}

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

// More than 128 clients: v = 0 the LDS-tile radix select, v = 1 the
// lane-group register sort with 128 values per lane (shipped), v = 2 the same
// with 64 values per lane and twice the lanes; for K <= 128: v = 4 the
// shipped one-lane pruned network, v = 3 two lanes of 64
extern "C" int median_big_probe(int v, const void* src, int K, int64_t N, void* out, void* stream) {
  auto s = reinterpret_cast<const float* const*>(src);
  auto o = reinterpret_cast<float*>(out);
  auto st = reinterpret_cast<hipStream_t>(stream);
  if (K > 1024 || N <= 0) return -1;
  if (v == 3) return K <= 128 ? launch_median_lanes<2, 64>(s, K, N, o, st) : -1;  // K <= 128, two lanes
  if (v == 4) return K <= 128 ? launch_median<128>(s, K, N, o, st) : -1;         // K <= 128, shipped
  if (K <= 128) return -1;
  if (v == 0) {
    if (K <= 256) return launch_median_radix<256>(s, K, N, o, st);
    if (K <= 512) return launch_median_radix<512>(s, K, N, o, st);
    return launch_median_radix<1024>(s, K, N, o, st);
  }
  if (v == 1) {
    if (K <= 256) return launch_median_lanes<2, 128>(s, K, N, o, st);
    if (K <= 512) return launch_median_lanes<4, 128>(s, K, N, o, st);
    return launch_median_lanes<8, 128>(s, K, N, o, st);
  }
  if (v == 2) {
    if (K <= 256) return launch_median_lanes<4, 64>(s, K, N, o, st);
    if (K <= 512) return launch_median_lanes<8, 64>(s, K, N, o, st);
    return launch_median_lanes<16, 64>(s, K, N, o, st);
  }
  // v == 5 / 6: the shipped layouts with 128- / 64-lane blocks
  if (v == 5) {
    if (K <= 256) return launch_median_lanes<4, 64, MedF32, 128>(s, K, N, o, st);
    if (K <= 512) return launch_median_lanes<4, 128, MedF32, 128>(s, K, N, o, st);
    return launch_median_lanes<8, 128, MedF32, 128>(s, K, N, o, st);
  }
  if (K <= 256) return launch_median_lanes<4, 64, MedF32, 64>(s, K, N, o, st);
  if (K <= 512) return launch_median_lanes<4, 128, MedF32, 64>(s, K, N, o, st);
  return launch_median_lanes<8, 128, MedF32, 64>(s, K, N, o, st);
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
