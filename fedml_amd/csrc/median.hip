// median.hip — gfx950 kernels for FedML's coordinate-wise median defense
// (core/security/defense/coordinate_wise_median_defense.py:24-32), exported
// through include/fedagg.h (fedagg_median, fedagg_median_f32) and linked into
// libfedagg.so beside fedagg.hip and robust.hip.  Its own translation unit so
// that the selection kernels rebuild without the reduction kernels.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <string>
#include <type_traits>
#include <utility>

#include "../../include/fedagg.h"

// 1 would keep the mirrored-pair merge (a lane select per cross-lane step) in
// the packed 4-lane kernels; 0 since round 4 (NOTES.md §5b)
constexpr int kPk16Mirror = 0;
// reversed DPP reads issued per batch in lanes4_merge_median
constexpr int kPk16Batch = 2;
// Loads of the lane-group kernels: a wave instruction reads 64 B of each of P
// rows' 128-B lines and the block's next wave reads the other half, so plain
// loads (0) keep the line in L2 for it; non-temporal ones (1) fetched 1.04-1.5x
// the algorithmic bytes vs 1.00-1.03x, at the same time
// (profiles/r03/lanes_nt/)
constexpr int kLanesNT = 0;
// Loads of the one-lane-per-column kernels (K <= 128; 256 B per wave
// instruction): 1 non-temporal, 0 plain
constexpr int kColsNT = 1;

extern "C" int fedagg_set_error_internal(int code, const char* msg);

namespace {

int set_error(int code, const std::string& msg) { return fedagg_set_error_internal(code, msg.c_str()); }

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(static_cast<int>(e), std::string(what) + ": " + hipGetErrorString(e));
  return FEDAGG_OK;
}

// Client rows arrive through pointer tables, which hipcc cannot prove are
// global memory (see fedagg.hip): the cast keeps the loads global, not FLAT.
template <class T>
__device__ __forceinline__ const T __attribute__((address_space(1)))* as_global(const T* p) {
  return (const T __attribute__((address_space(1)))*)(p);
}

// loads of the lane-group kernels (kLanesNT)
template <class T>
__device__ __forceinline__ T lanes_load(const T __attribute__((address_space(1)))* p) {
  if constexpr (kLanesNT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}
// loads of the one-lane-per-column kernels (kColsNT)
template <class T>
__device__ __forceinline__ T cols_load(const T __attribute__((address_space(1)))* p) {
  if constexpr (kColsNT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

// ---------------------------------------------------------------------------
// Coordinate-wise median (the reference's "wise_median" defense:
// core/security/defense/coordinate_wise_median_defense.py:24-32, i.e.
// torch.median(stack, dim=-1).values: the LOWER median, element (K-1)/2 of the
// sorted column; any NaN in the column makes the result that NaN).
//
// One lane per parameter element holds the column's K values in registers
// (KMAX >= K slots).  The column is padded with -inf / +inf so that its lower
// median always lands at the network's fixed middle slot (KMAX-1)/2; a
// pairwise sorting network is then fully unrolled at compile time, and since
// only that one output slot is used, the compiler deletes every comparator
// that does not feed it.  Loads are 4 B per lane (256 B per wave
// instruction), all K of them independent and in flight together.  K == KMAX
// (e.g. 128 clients) gets a kernel with no padding logic at all.
//
// VALU per element at K = 128 (gfx950 ISA): 2,017 v_min/v_max (+61 fused
// min3/max3), 128 NaN compares; ~3,470 with the earlier Batcher network,
// per-client 64-bit addressing and in-line first-NaN tracking.

__device__ __forceinline__ void cmpx(float& a, float& b) {
  const float lo = fminf(a, b), hi = fmaxf(a, b);
  a = lo;
  b = hi;
}

// Parberry's pairwise sorting network on N slots, generated at compile time.
// Pruned to the one output slot the median needs, it keeps 2,011 min/max at
// N = 128 where Batcher's odd-even merge sort keeps 2,299 (same 1,471
// comparators before pruning; the pairwise network's last stages feed fewer
// slots).
struct CmpPair {
  int a, b;
};
template <int N>
struct PairwiseNet {
  // emit(a, b) for every comparator in network order; returns the count
  template <class F>
  static constexpr int walk(F emit) {
    int m = 0;
    int a = 1;
    for (; a < N; a *= 2) {
      int b = a, c = 0;
      while (b < N) {
        emit(m++, b - a, b);
        ++b;
        c = (c + 1) % a;
        if (c == 0) b += a;
      }
    }
    a /= 4;
    for (int e = 1; a > 0; a /= 2, e = e * 2 + 1) {
      for (int d = e; d > 0; d /= 2) {
        int b = (d + 1) * a, c = 0;
        while (b < N) {
          emit(m++, b - d * a, b);
          ++b;
          c = (c + 1) % a;
          if (c == 0) b += a;
        }
      }
    }
    return m;
  }
  static constexpr int M = walk([](int, int, int) {});
  struct Table {
    CmpPair p[M > 0 ? M : 1];
  };
  static constexpr Table make() {
    Table t{};
    walk([&t](int m, int x, int y) { t.p[m] = CmpPair{x, y}; });
    return t;
  }
  static constexpr Table table = make();
};

// two 16-bit order keys per register: one v_pk_min_i16 + one v_pk_max_i16
typedef short short2_t __attribute__((ext_vector_type(2)));
typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void cmpx(short2_t& a, short2_t& b) {
  const short2_t lo = __builtin_elementwise_min(a, b), hi = __builtin_elementwise_max(a, b);
  a = lo;
  b = hi;
}

template <int N, int I, class T>
__device__ __forceinline__ void net_cmp(T (&v)[N]) {
  constexpr int A = PairwiseNet<N>::table.p[I].a, B = PairwiseNet<N>::table.p[I].b;
  cmpx(v[A], v[B]);
}
template <int N, class T, int... I>
__device__ __forceinline__ void net_apply(T (&v)[N], std::integer_sequence<int, I...>) {
  (net_cmp<N, I>(v), ...);
}
template <int N, class T>
__device__ __forceinline__ void pairwise_sort(T (&v)[N]) {
  net_apply<N, T>(v, std::make_integer_sequence<int, PairwiseNet<N>::M>{});
}

// Element types of the median kernels.  Every column value becomes an fp32
// "selection value" whose float order is the element's order, the networks
// select on those, and the selected value maps back to the input's bits
// exactly (it is one of the inputs).  fp32 and bf16 widen exactly (bf16 is
// the top half of an fp32).  f16 maps to an order-preserving 16-bit key
// placed in the mantissa of [1, 2): x ^ 0x8000 for positive, ~x for negative
// values, so -inf < -finite < -0 < +0 < +finite < +inf as keys, all normal
// floats, and the ±inf pads stay below / above every key.  (Widening f16 to
// fp32 with v_cvt kept both forms live and took the K = 128 kernel to 256
// VGPRs, occupancy 1.)  nan() tests a selection value for NaN.
struct MedF32 {
  using S = float;
  static __device__ __forceinline__ float widen(S x) { return x; }
  static __device__ __forceinline__ S narrow(float v) { return v; }
  static __device__ __forceinline__ bool nan(float v) { return __builtin_isnan(v); }
  static __device__ __forceinline__ bool raw_nan(S x) { return __builtin_isnan(x); }
  static constexpr bool kReloadNan = false;
  // running "any NaN so far" over the column's selection values
  using NanAcc = bool;
  static __device__ __forceinline__ void nan_add(NanAcc& a, float v) { a |= __builtin_isnan(v); }
  static __device__ __forceinline__ bool nan_any(NanAcc a) { return a; }
  static constexpr uint32_t kNegInf = 0xff800000u, kPosInf = 0x7f800000u;
};
struct IsNanAcc {
  using NanAcc = bool;
  static __device__ __forceinline__ void nan_add(NanAcc& a, float v) { a |= __builtin_isnan(v); }
  static __device__ __forceinline__ bool nan_any(NanAcc a) { return a; }
};
struct MedBF16 : IsNanAcc {
  using S = uint16_t;
  static __device__ __forceinline__ bool raw_nan(S x) { return (x & 0x7fffu) > 0x7f80u; }
  static constexpr bool kReloadNan = true;
  static __device__ __forceinline__ float widen(S x) { return __uint_as_float(uint32_t(x) << 16); }
  static __device__ __forceinline__ S narrow(float v) { return S(__float_as_uint(v) >> 16); }
  static __device__ __forceinline__ bool nan(float v) { return __builtin_isnan(v); }
  static constexpr uint32_t kNegInf = 0xff80u, kPosInf = 0x7f80u;
};
struct MedF16 {
  using S = uint16_t;
  static __device__ __forceinline__ bool raw_nan(S x) { return (x & 0x7fffu) > 0x7c00u; }
  static constexpr bool kReloadNan = true;
  // The value arrives in the high half (as bf16 does: a d16_hi load), its
  // order key is built there (x ^ 0x8000 for positive, ~x for negative values)
  // and shifted down two bits: a positive float below 2.0 whose float order
  // is the key order (normal for every non-NaN key: -inf's key 0x03ff gives
  // 0x00ffc000).
  static __device__ __forceinline__ float widen(S x) {
    const uint32_t u = uint32_t(x) << 16;
    const uint32_t neg = uint32_t(int32_t(u) >> 31);
    return __uint_as_float((u ^ (0x80000000u | (neg & 0x7fff0000u))) >> 2);
  }
  static __device__ __forceinline__ S narrow(float v) {
    const uint32_t k = (__float_as_uint(v) << 2) >> 16;  // the 16-bit key
    const uint32_t neg = ~uint32_t(int32_t(k << 16) >> 31);  // key below 0x8000: a negative value
    return S(k ^ ((neg & 0x7fffu) | 0x8000u));
  }
  static __device__ __forceinline__ uint32_t key(float v) { return (__float_as_uint(v) << 2) >> 16; }
  // NaN keys: +NaN 0x7c01..0x7fff -> 0xfc01..0xffff, -NaN 0xfc01..0xffff -> 0x0000..0x03fe
  static __device__ __forceinline__ bool nan(float v) {
    const uint32_t k = key(v);
    return __float_as_uint(v) < 0x40000000u && (k > 0xfc00u || k < 0x03ffu);
  }
  // rotated key (k - 0x3ff) mod 2^16: NaN keys land above 0xf801, every other
  // key at or below it, so one unsigned compare per value
  using NanAcc = bool;
  static __device__ __forceinline__ void nan_add(NanAcc& a, float v) { a |= ((key(v) - 0x3ffu) & 0xffffu) > 0xf801u; }
  static __device__ __forceinline__ bool nan_any(NanAcc a) { return a; }
  static constexpr uint32_t kNegInf = 0xfc00u, kPosInf = 0x7c00u;
};

// -inf / +inf in each element type: what a padded slot's load returns
template <class E>
__device__ typename E::S g_median_pad[2] = {__builtin_bit_cast(typename E::S, static_cast<std::conditional_t<
                                                sizeof(typename E::S) == 4, uint32_t, uint16_t>>(E::kNegInf)),
                                            __builtin_bit_cast(typename E::S, static_cast<std::conditional_t<
                                                sizeof(typename E::S) == 4, uint32_t, uint16_t>>(E::kPosInf))};

// Row base of client row p for a launch starting at column col0 (> 0 only
// past 2^30 columns): an opaque SGPR pair, so the loads keep the
// SGPR-base + 32-bit VGPR-offset form (left visible, the compiler folds col0
// into a per-lane 64-bit address: 2.2x slower at K = 128).
template <class T>
__device__ __forceinline__ const char __attribute__((address_space(1)))* row_base(const T* p, int64_t col0) {
  uint64_t b = reinterpret_cast<uint64_t>(p) + uint64_t(col0) * sizeof(T);
  asm("" : "+s"(b));
  return reinterpret_cast<const char __attribute__((address_space(1)))*>(b);
}

// Columns [col0, col0 + N) of the rows; out points at column col0's slot.
// Launches cover at most 2^30 columns (kMedianChunk) so that a lane's byte
// offset from the (wave-uniform) row base + col0 fits in 32 bits.
template <int KMAX, bool FULL, int BS, bool PRIO = false, class E = MedF32, bool OFF = false>
__global__ __launch_bounds__(BS) void median_kernel(const typename E::S* const* __restrict__ src, int K, int64_t N,
                                                    typename E::S* __restrict__ out, int64_t col0 = 0) {
  const int64_t e = int64_t(blockIdx.x) * BS + threadIdx.x;
  if constexpr (FULL) K = KMAX;  // K == KMAX: no padding, no per-client conditions
  const int below = (KMAX - 1) / 2 - (K - 1) / 2;  // -inf pads; the rest of the padding is +inf
  // K < KMAX: the KMAX slot pointers (pads point at a ±inf constant) staged
  // in LDS once per block.  Read per slot at a wave-uniform address and moved
  // to SGPRs, they keep the loads in the SGPR-base form and batched; reading
  // src[min(c, K - 1)] instead issued one s_load per client and waited for
  // each (2.3x the K == KMAX time at K = 100).
  __shared__ const typename E::S* tab[FULL ? 1 : KMAX];
  if constexpr (!FULL) {
    for (int i = threadIdx.x; i < KMAX; i += BS) tab[i] = i < K ? src[i] : &g_median_pad<E>[i - K < below ? 0 : 1];
    __syncthreads();
  }
  if (e >= N) return;
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);  // issue this wave's loads ahead of others' sorting
  // The host guarantees N * 4 < 2^32: a 32-bit byte offset on each
  // wave-uniform row base lets every load use the SGPR-base + VGPR-offset
  // form, with no per-client 64-bit address arithmetic on the VALU.
  const uint32_t boff = uint32_t(e) * uint32_t(sizeof(typename E::S));
  float v[KMAX];
  typename E::NanAcc nacc{};
#pragma unroll
  for (int c = 0; c < KMAX; ++c) {
    // Keep at most 16 row pointers live in SGPRs: without the barrier the
    // scheduler hoists all K pointer loads to the top and spills them.
    if (c % 16 == 0 && c) __builtin_amdgcn_sched_barrier(0);
    // A padded slot (c >= K) reads a ±inf constant: its row pointer is the
    // pad and its lane offset is 0, so the load itself yields the pad.
    // Nothing per slot waits for a load here: all KMAX loads are in flight
    // before the first value is used.
    const bool live = FULL || c < K;
    const typename E::S* p;
    if constexpr (FULL) {
      p = src[c];
    } else {
      // readfirstlane returns int: go through uint32_t, or a low word with
      // its top bit set sign-extends over the high word
      const uint64_t t = reinterpret_cast<uint64_t>(tab[c]);
      const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(t >> 32))));
      const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(t))));
      p = reinterpret_cast<const typename E::S*>((uint64_t(hi) << 32) | uint64_t(lo));
    }
    const char __attribute__((address_space(1)))* row;
    if constexpr (OFF)
      row = live ? row_base(p, col0) : reinterpret_cast<const char __attribute__((address_space(1)))*>(as_global(p));
    else
      row = reinterpret_cast<const char __attribute__((address_space(1)))*>(as_global(p));
    v[c] = E::widen(cols_load(
        reinterpret_cast<const typename E::S __attribute__((address_space(1)))*>(row + (live ? boff : 0u))));
    if constexpr (sizeof(typename E::S) == 2) E::nan_add(nacc, v[c]);
  }
  // torch returns the first NaN of the column (client order) if there is
  // one; the common case pays one test per client.  fp32 tests after every
  // load is in flight (testing inside the load loop waited for each pair of
  // loads); 16-bit rows test as they widen (with all loads in flight first,
  // the raw and widened values are both live: 259 VGPRs; this kernel is
  // their unaligned-row path, the packed kernel takes aligned rows).
  // Pads are ±inf, never NaN.
  if constexpr (sizeof(typename E::S) == 4) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < KMAX; ++c) E::nan_add(nacc, v[c]);
  }
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  // Only a lane holding a NaN column searches.  fp32 tests the registers (one
  // unordered compare); for 16-bit rows that search got speculated above the
  // branch and kept both the loaded and the widened values live (259-267
  // VGPRs), so they re-read the column in client order (cache hits).
  typename E::S nan_raw{};
  const bool has_nan = E::nan_any(nacc);
  if (has_nan) {
    if constexpr (E::kReloadNan) {
#pragma unroll 1
      for (int c = 0; c < K; ++c) {
        const auto row = row_base(src[c], col0);
        const typename E::S r = *reinterpret_cast<const typename E::S __attribute__((address_space(1)))*>(row + boff);
        if (E::raw_nan(r)) {
          nan_raw = r;
          break;
        }
      }
    } else {
      float nan_v = 0.f;
      bool found = false;
#pragma unroll
      for (int c = 0; c < KMAX; ++c) {
        const bool n = (FULL || c < K) && !found && E::nan(v[c]);
        nan_v = n ? v[c] : nan_v;
        found = found || n;
      }
      nan_raw = E::narrow(nan_v);
    }
  }
  pairwise_sort<KMAX>(v);
  out[e] = has_nan ? nan_raw : E::narrow(v[(KMAX - 1) / 2]);
}

constexpr int64_t kMedianChunk = int64_t(1) << 30;  // columns per launch of the 32-bit-offset kernels

template <int KMAX, class E = MedF32>
int launch_median(const typename E::S* const* src, int K, int64_t N, typename E::S* out, hipStream_t st) {
  constexpr int BS = 64;  // 3 % faster than 256 at config 3 (tools/median_probe.py, two boxes)
  for (int64_t c0 = 0; c0 < N; c0 += kMedianChunk) {
    const int64_t n = N - c0 < kMedianChunk ? N - c0 : kMedianChunk;
    const int64_t grid = (n + BS - 1) / BS;
    if (K == KMAX && c0 == 0)
      hipLaunchKernelGGL((median_kernel<KMAX, true, BS, false, E>), dim3(unsigned(grid)), dim3(BS), 0, st, src, K, n,
                         out, c0);
    else if (c0 == 0)
      hipLaunchKernelGGL((median_kernel<KMAX, false, BS, false, E>), dim3(unsigned(grid)), dim3(BS), 0, st, src, K, n,
                         out, c0);
    else  // past 2^30 columns: the padded kernel (correct for K == KMAX too) with the row offset
      hipLaunchKernelGGL((median_kernel<KMAX, false, BS, false, E, true>), dim3(unsigned(grid)), dim3(BS), 0, st, src,
                         K, n, out + c0, c0);
  }
  return check_launch("fedagg_median");
}

// 16-bit rows, K <= 128, two columns per lane: a 32-bit load brings columns
// 2e and 2e+1 of a client as one register, each half is turned into an
// order-preserving int16 key (x ^ 0x7fff for negative values, so signed
// compares follow the float order, -0 just below +0), and the same pruned
// network runs on v_pk_min_i16 / v_pk_max_i16: half the VALU per column of the
// widening kernel, which is VALU-bound on 16-bit rows.  Keys map back to the
// input bits by the same transform.  Pads are the int16 extremes, below / above
// every non-NaN key; a NaN column returns its first NaN, as everywhere.  Needs
// 4-byte aligned rows and output (the FEDAGG_ALIGNED16 flag); an odd last
// column is loaded and stored as 16 bits by its lane.
__device__ __forceinline__ short2_t pk16_key(uint32_t x) {
  const short2_t v = __builtin_bit_cast(short2_t, x);
  return v ^ ((v >> short(15)) & short(0x7fff));
}
__device__ __forceinline__ uint32_t pk16_bits(short2_t k) {
  return __builtin_bit_cast(uint32_t, k ^ ((k >> short(15)) & short(0x7fff)));
}

template <int KMAX, bool FULL, class E, bool TAIL, bool OFF>
__device__ __forceinline__ void median_pk16_pair(const uint16_t* const* __restrict__ src, int K, int64_t e,
                                                 uint16_t* __restrict__ out, int64_t col0) {
  if constexpr (FULL) K = KMAX;
  const uint32_t boff = uint32_t(e) * 4u;
  const int below = (KMAX - 1) / 2 - (K - 1) / 2;
  uint32_t raw[KMAX];
  uint32_t nanacc = 0;  // per half, max of |x| bits
#pragma unroll
  for (int c = 0; c < KMAX; ++c) {
    if (c % 16 == 0 && c) __builtin_amdgcn_sched_barrier(0);
    const int ci = (FULL || c < K) ? c : K - 1;
    const char __attribute__((address_space(1)))* row;
    if constexpr (OFF)
      row = row_base(src[ci], col0);
    else
      row = reinterpret_cast<const char __attribute__((address_space(1)))*>(as_global(src[ci]));
    uint32_t x;
    if constexpr (!TAIL)
      x = cols_load(reinterpret_cast<const uint32_t __attribute__((address_space(1)))*>(row + boff));
    else  // the odd last column alone, duplicated into both halves
      x = *reinterpret_cast<const uint16_t __attribute__((address_space(1)))*>(row + boff) * 0x10001u;
    raw[c] = x;
  }
  __builtin_amdgcn_sched_barrier(0);  // every load in flight before the first test (see median_kernel)
#pragma unroll
  for (int c = 0; c < KMAX; ++c) {
    const uint32_t mag = raw[c] & 0x7fff7fffu;
    nanacc = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(ushort2_t, nanacc),
                                                                     __builtin_bit_cast(ushort2_t, mag)));
  }
  const bool nan_lo = (nanacc & 0xffffu) > E::kPosInf, nan_hi = (nanacc >> 16) > E::kPosInf;
  uint32_t nan_bits = 0;
  if (nan_lo || nan_hi) {  // first NaN per half, in client order (only columns holding one)
    bool f_lo = false, f_hi = false;
#pragma unroll
    for (int c = 0; c < KMAX; ++c) {
      // predicated, not `break`: a data-dependent exit stops the full unroll
      // and puts raw[] in scratch (272-528 B/lane before)
      const bool live = FULL || c < K;
      const uint32_t x = raw[c];
      const bool n_lo = live && !f_lo && (x & 0x7fffu) > E::kPosInf;
      const bool n_hi = live && !f_hi && ((x >> 16) & 0x7fffu) > E::kPosInf;
      if (n_lo) nan_bits = (nan_bits & 0xffff0000u) | (x & 0xffffu);
      if (n_hi) nan_bits = (nan_bits & 0xffffu) | (x & 0xffff0000u);
      f_lo = f_lo || n_lo;
      f_hi = f_hi || n_hi;
    }
  }
  short2_t v[KMAX];
#pragma unroll
  for (int c = 0; c < KMAX; ++c) {
    if constexpr (FULL)
      v[c] = pk16_key(raw[c]);
    else
      v[c] = (c < K) ? pk16_key(raw[c]) : ((c - K < below) ? short2_t(short(-32768)) : short2_t(short(32767)));
  }
  pairwise_sort<KMAX>(v);
  uint32_t m = pk16_bits(v[(KMAX - 1) / 2]);
  if (nan_lo) m = (m & 0xffff0000u) | (nan_bits & 0xffffu);
  if (nan_hi) m = (m & 0xffffu) | (nan_bits & 0xffff0000u);
  if constexpr (!TAIL)
    *reinterpret_cast<uint32_t*>(out + 2 * e) = m;
  else
    out[2 * e] = uint16_t(m);
}

template <int KMAX, bool FULL, class E, int BS = 256, bool OFF = false>
__global__ __launch_bounds__(BS) void median_pk16_kernel(const uint16_t* const* __restrict__ src, int K, int64_t N,
                                                         uint16_t* __restrict__ out, int64_t col0) {
  static_assert(sizeof(typename E::S) == 2, "16-bit rows");
  const int64_t e = int64_t(blockIdx.x) * BS + threadIdx.x;  // column pair
  const int64_t pairs = (N + 1) / 2;
  if (e >= pairs) return;
  if ((N & 1) && e == pairs - 1)
    median_pk16_pair<KMAX, FULL, E, true, OFF>(src, K, e, out, col0);
  else
    median_pk16_pair<KMAX, FULL, E, false, OFF>(src, K, e, out, col0);
}

template <int KMAX, class E>
int launch_median_pk16(const uint16_t* const* src, int K, int64_t N, uint16_t* out, hipStream_t st) {
  constexpr int BS = 64;
  for (int64_t c0 = 0; c0 < N; c0 += kMedianChunk) {  // even chunk starts: 4-byte pairs stay aligned
    const int64_t n = N - c0 < kMedianChunk ? N - c0 : kMedianChunk;
    const int64_t grid = ((n + 1) / 2 + BS - 1) / BS;
    if (K == KMAX && c0 == 0)
      hipLaunchKernelGGL((median_pk16_kernel<KMAX, true, E, BS>), dim3(unsigned(grid)), dim3(BS), 0, st, src, K, n,
                         out, c0);
    else if (c0 == 0)
      hipLaunchKernelGGL((median_pk16_kernel<KMAX, false, E, BS>), dim3(unsigned(grid)), dim3(BS), 0, st, src, K, n,
                         out, c0);
    else
      hipLaunchKernelGGL((median_pk16_kernel<KMAX, false, E, BS, true>), dim3(unsigned(grid)), dim3(BS), 0, st, src,
                         K, n, out + c0, c0);
  }
  return check_launch("fedagg_median");
}

// More than 128 clients, in registers: P adjacent lanes share one column,
// each holding R of its KMAX = P·R (±inf-padded) values, slot s = sub·R + j =
// client s (shipped: P = 4, R = 64 up to 256 clients, then R = 128 with P = 4,
// 8, 16 or 32, i.e. up to 4096 clients).  Every lane sorts its R values with the pairwise network (all outputs
// used, so nothing is pruned); the sorted runs are then merged across lanes as
// in a bitonic merge sort:
//   - "reverse pairing" of two sorted runs A, B of length L held by lane
//     groups g and g ^ (G-1): element i of A meets element L-1-i of B, the
//     lower group keeps the min (the L smallest, a bitonic sequence), the
//     upper the max.  Partner lane = sub ^ (G-1), partner register = R-1-i;
//   - a half-cleaner cascade sorts each bitonic half: stages whose slot
//     distance is a multiple of R pair lane sub with sub ^ m at the same
//     register, the rest run inside the lane.
// Cross-lane moves are single DPP movs (xor 1 / 2 / 3 quad permutes, xor 7 =
// row_half_mirror, xor 15 = row_mirror), the min-or-max choice one v_med3
// against ±inf.  The last level needs no merge: after its reverse pairing the
// lower half holds exactly the KMAX/2 smallest values, whose maximum sits at
// the padded median slot KMAX/2 - 1, i.e. it is the column's lower median.
// VALU per column ≈ 8k (P·R = 4·64), 20k (4·128), 49k (8·128) lane-ops,
// against 2k for K <= 128.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ short2_t dpp_mov(short2_t x) {
  return __builtin_bit_cast(short2_t, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
template <int M>
constexpr int dpp_xor_ctrl() {
  static_assert(M == 1 || M == 2 || M == 3 || M == 7 || M == 15, "lane xor pattern without a single DPP mov");
  // quad_perm [1,0,3,2], [2,3,0,1], [3,2,1,0]; row_half_mirror; row_mirror
  return M == 1 ? 0xB1 : M == 2 ? 0x4E : M == 3 ? 0x1B : M == 7 ? 0x141 : 0x140;
}

// The value of lane ^ M: one DPP mov where a pattern exists (xor 1, 2, 3,
// 7, 15), two for xor 4 (xor 7 then xor 3), else ds_bpermute (xor 31: the
// last level of the 32-lane groups above 2,048 clients).
template <int M>
constexpr bool dpp_xor_ok() { return M == 1 || M == 2 || M == 3 || M == 7 || M == 15; }
template <int M>
__device__ __forceinline__ float xor_mov(float x) {
  if constexpr (dpp_xor_ok<M>()) return dpp_mov<dpp_xor_ctrl<M>()>(x);
  else if constexpr (M == 4) return dpp_mov<dpp_xor_ctrl<3>()>(dpp_mov<dpp_xor_ctrl<7>()>(x));  // (i ^ 7) ^ 3
  else return __int_as_float(__shfl_xor(__float_as_int(x), M, 64));
}

// min (lower lanes, sel = -inf) or max (upper lanes, sel = +inf) of own
// register i and the partner lane's register R-1-i, for every i
template <int M, int R>
__device__ __forceinline__ void lanes_reverse_pair(float (&v)[R], float sel) {
  // opaque to the compiler: knowing sel is ±inf it splits every v_med3 into
  // min, max and a select (three ops and twice the live registers)
  asm volatile("" : "+v"(sel));
#pragma unroll
  for (int i = 0; i < R / 2; ++i) {
    const float a = xor_mov<M>(v[R - 1 - i]);
    const float b = xor_mov<M>(v[i]);
    v[i] = __builtin_amdgcn_fmed3f(v[i], a, sel);
    v[R - 1 - i] = __builtin_amdgcn_fmed3f(v[R - 1 - i], b, sel);
  }
}

// half-cleaner stage between lanes sub and sub ^ M, same register
template <int M, int R>
__device__ __forceinline__ void lanes_cross_stage(float (&v)[R], int sub) {
  float sel = (sub & M) ? __builtin_huge_valf() : -__builtin_huge_valf();
  asm volatile("" : "+v"(sel));
#pragma unroll
  for (int i = 0; i < R; ++i) v[i] = __builtin_amdgcn_fmed3f(v[i], xor_mov<M>(v[i]), sel);
}

// in-lane half-cleaner cascade: a bitonic register array -> ascending
template <int R>
__device__ __forceinline__ void lane_bitonic_merge(float (&v)[R]) {
#pragma unroll
  for (int d = R / 2; d > 0; d /= 2) {
#pragma unroll
    for (int i = 0; i < R; ++i)
      if ((i & d) == 0) cmpx(v[i], v[i + d]);
  }
}

// merge levels G = 2, 4, 8 (< P): afterwards every group of G lanes holds its
// G·R values sorted ascending over slots (sub % G)·R + j
template <int G, int P, int R>
__device__ __forceinline__ void lanes_merge_levels(float (&v)[R], int sub) {
  if constexpr (G < P) {
    static_assert(G <= 16, "lane groups of at most 32");
    lanes_reverse_pair<G - 1>(v, (sub & (G / 2)) ? __builtin_huge_valf() : -__builtin_huge_valf());
    if constexpr (G == 16) lanes_cross_stage<4>(v, sub);  // slot distance 4R
    if constexpr (G >= 8) lanes_cross_stage<2>(v, sub);  // slot distance 2R
    if constexpr (G >= 4) lanes_cross_stage<1>(v, sub);  // slot distance R
    lane_bitonic_merge(v);
    lanes_merge_levels<G * 2, P, R>(v, sub);
  }
}

// Four lanes per column (P = 4), odd lanes in the reversed order
// (complemented int16 keys), every lane's run sorted ascending in its own
// order.  Lanes 2q and 2q + 1 hold runs A (ascending) and B (descending
// in the true order), so A and B form a bitonic sequence whose half-cleaner
// pairs register i with register i: the even lane keeps min(a, b) and the odd
// lane max(a, b), which in its reversed order is min(own, rev(partner)) too.
// An in-lane half-cleaner cascade then sorts each lane.  Lanes 0 and 1 now
// hold the sorted 2R-run X (lane 0 ascending, lane 1 descending), lanes 2
// and 3 the run Y.  The 2R smallest of X and Y are min(X[i], Y[2R-1-i]),
// i.e. lane 0's register i against lane 3's register i and lane 2's against
// lane 1's: the lower median is the max of min(own, rev(partner ^ 3)) over
// lanes 0 and 2 (lanes 1 and 3 compute the same expression, unused).
// Per register: one v_not_b32_dpp and one v_pk_min_i16 per level, against a
// DPP mov, v_pk_min, v_pk_max and a lane select before.  (fp32 keeps the
// mirrored pairing: a negated DPP read cannot fuse into an IEEE min there,
// and its min-or-max is already one v_med3 against ±inf.)
[[maybe_unused]] __device__ __forceinline__ short2_t lanes_rev(short2_t x) { return ~x; }
[[maybe_unused]] __device__ __forceinline__ short2_t lanes_min(short2_t a, short2_t b) {
  return __builtin_elementwise_min(a, b);
}
[[maybe_unused]] __device__ __forceinline__ short2_t lanes_max(short2_t a, short2_t b) {
  return __builtin_elementwise_max(a, b);
}

template <class T, int R>
__device__ __forceinline__ T lanes4_merge_median(T (&v)[R]) {
  constexpr int B = kPk16Batch;  // reversed reads in batches: none right behind its register's write
#pragma unroll
  for (int i0 = 0; i0 < R; i0 += B) {
    T t[B];
#pragma unroll
    for (int k = 0; k < B; ++k) t[k] = lanes_rev(dpp_mov<dpp_xor_ctrl<1>()>(v[i0 + k]));
#pragma unroll
    for (int k = 0; k < B; ++k) v[i0 + k] = lanes_min(v[i0 + k], t[k]);
  }
#pragma unroll
  for (int d = R / 2; d > 0; d /= 2) {
#pragma unroll
    for (int i = 0; i < R; ++i)
      if ((i & d) == 0) cmpx(v[i], v[i + d]);
  }
  T m = lanes_min(v[0], lanes_rev(dpp_mov<dpp_xor_ctrl<3>()>(v[0])));
#pragma unroll
  for (int i0 = 0; i0 < R; i0 += B) {
    T t[B];
#pragma unroll
    for (int k = 0; k < B; ++k) t[k] = lanes_rev(dpp_mov<dpp_xor_ctrl<3>()>(v[i0 + k]));
#pragma unroll
    for (int k = (i0 == 0); k < B; ++k) m = lanes_max(m, lanes_min(v[i0 + k], t[k]));
  }
  return lanes_max(m, dpp_mov<dpp_xor_ctrl<2>()>(m));  // lane 0: its max and lane 2's
}

template <int P, int R, bool FULL, class E = MedF32, int BS = 256>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(2))) void median_lanes_kernel(
    const typename E::S* const* __restrict__ src, int K, int64_t N, typename E::S* __restrict__ out) {
  using S = typename E::S;
  static_assert(P == 2 || P == 4 || P == 8 || P == 16 || P == 32, "2 to 32 lanes per column");
  static_assert(R == 64 || R == 128, "64 or 128 values per lane");
  constexpr int KMAX = P * R, PAD = 2;
  // Row pointer of every slot, skewed by PAD entries per lane group so the P
  // lanes of a column read different LDS banks.  A padded slot (K < KMAX)
  // points at a ±inf constant and its column offset is masked to 0, so the
  // load itself yields the pad: no per-slot, per-lane select.
  __shared__ const S* rows[KMAX + PAD * P];
  __shared__ uint64_t offmask[FULL ? 1 : KMAX + PAD * P];
  const int t = threadIdx.x, sub = t & (P - 1);
  if constexpr (FULL) K = KMAX;
  const int below = KMAX / 2 - 1 - (K - 1) / 2;  // -inf pads; the rest of the padding is +inf
  for (int i = t; i < KMAX; i += BS) {
    const int q = i + PAD * (i / R);
    if (FULL || i < K) {
      rows[q] = src[i];
      if constexpr (!FULL) offmask[q] = ~uint64_t(0);
    } else {
      rows[q] = &g_median_pad<E>[i - K < below ? 0 : 1];
      offmask[q] = 0;
    }
  }
  __syncthreads();
  // every lane stays active through the DPP exchanges; a column past the end
  // recomputes the last one and does not store
  const int64_t e = (int64_t(blockIdx.x) * BS + t) / P;
  const uint64_t boff = uint64_t(e < N ? e : N - 1) * sizeof(S);
  float v[R];
  typename E::NanAcc nacc{};
#pragma unroll
  for (int j = 0; j < R; ++j) {
    if (j % 16 == 0 && j) __builtin_amdgcn_sched_barrier(0);
    const int q = sub * (R + PAD) + j;
    const uint64_t off = FULL ? boff : (boff & offmask[q]);
    const auto row = reinterpret_cast<const char*>(rows[q]);
    v[j] = E::widen(lanes_load(as_global(reinterpret_cast<const S*>(row + off))));
  }
  __builtin_amdgcn_sched_barrier(0);  // every load in flight before the first test (see median_kernel)
#pragma unroll
  for (int j = 0; j < R; ++j) E::nan_add(nacc, v[j]);
  const bool has_nan = E::nan_any(nacc);
  // first NaN of the column in client (= slot) order, only in waves holding
  // one (pads are ±inf, never NaN)
  int nan_slot = KMAX;
  S nan_raw{};
  if (__ballot(has_nan)) {
    // re-read this lane's slots in client order (cache hits; see median_kernel)
#pragma unroll 1
    for (int j = 0; j < R; ++j) {
      const int q = sub * (R + PAD) + j;
      const uint64_t off = FULL ? boff : (boff & offmask[q]);
      const S r = *as_global(reinterpret_cast<const S*>(reinterpret_cast<const char*>(rows[q]) + off));
      if (E::raw_nan(r)) {
        nan_slot = sub * R + j;
        nan_raw = r;
        break;
      }
    }
#pragma unroll
    for (int m = 1; m < P; m <<= 1) {
      const int os = __shfl_xor(nan_slot, m, 64);
      using U = std::conditional_t<sizeof(S) == 4, uint32_t, uint16_t>;  // move the bits, not the value
      const S ov = __builtin_bit_cast(
          S, U(__shfl_xor(int(uint32_t(__builtin_bit_cast(U, nan_raw))), m, 64)));
      if (os < nan_slot) {
        nan_slot = os;
        nan_raw = ov;
      }
    }
  }
  pairwise_sort<R>(v);
  lanes_merge_levels<2, P, R>(v, sub);
  // last level: after the reverse pairing against sub ^ (P-1) the lower P/2
  // lanes hold the KMAX/2 smallest values; their max is the median
  lanes_reverse_pair<P - 1>(v, (sub & (P / 2)) ? __builtin_huge_valf() : -__builtin_huge_valf());
  float m = v[0];
#pragma unroll
  for (int i = 1; i < R; ++i) m = fmaxf(m, v[i]);
  if constexpr (P >= 4) m = fmaxf(m, dpp_mov<dpp_xor_ctrl<1>()>(m));
  if constexpr (P >= 8) m = fmaxf(m, dpp_mov<dpp_xor_ctrl<2>()>(m));
  if constexpr (P >= 16) m = fmaxf(m, dpp_mov<dpp_xor_ctrl<7>()>(m));  // quad maxima across the two quads
  if constexpr (P >= 32) m = fmaxf(m, dpp_mov<dpp_xor_ctrl<15>()>(m));  // the two 8-lane halves of a row
  if (sub == 0 && e < N) out[e] = nan_slot < KMAX ? nan_raw : E::narrow(m);
}

template <int P, int R, class E = MedF32, int BS = 256>
int launch_median_lanes(const typename E::S* const* src, int K, int64_t N, typename E::S* out, hipStream_t st) {
  const int64_t grid = (N * P + BS - 1) / BS;
  if (grid > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, "fedagg_median: N too large");
  if (K == P * R)
    hipLaunchKernelGGL((median_lanes_kernel<P, R, true, E, BS>), dim3(unsigned(grid)), dim3(BS), 0, st, src, K, N,
                       out);
  else
    hipLaunchKernelGGL((median_lanes_kernel<P, R, false, E, BS>), dim3(unsigned(grid)), dim3(BS), 0, st, src, K, N,
                       out);
  return check_launch("fedagg_median");
}

// 16-bit rows with more than 128 clients, two columns per register: the lane
// group layout above on the packed int16 order keys of median_pk16_pair.  One
// 32-bit load brings columns 2e and 2e+1 of a client; the in-lane sorts and
// half-cleaners are v_pk_min_i16 / v_pk_max_i16 (one op per comparator side
// for TWO columns), so the per-column VALU is about half of the widening
// kernel's, which is what bounds this range.  The cross-lane min-or-max has no
// packed med3: both sides and one v_cndmask on a lane mask.  Pads are packed
// ±inf (their keys sit below / above every non-NaN key); a NaN column returns
// its first NaN in client order, per half.  An odd last column runs as the
// TAIL instantiation: one block whose every column group recomputes the
// duplicated lone column, and lane 0 stores it.
template <int M>
__device__ __forceinline__ short2_t xor_mov(short2_t x) {
  if constexpr (dpp_xor_ok<M>()) return dpp_mov<dpp_xor_ctrl<M>()>(x);
  else if constexpr (M == 4) return dpp_mov<dpp_xor_ctrl<3>()>(dpp_mov<dpp_xor_ctrl<7>()>(x));
  else return __builtin_bit_cast(short2_t, __shfl_xor(__builtin_bit_cast(int, x), M, 64));
}
__device__ __forceinline__ short2_t pk_pick(short2_t a, short2_t b, bool up) {
  const short2_t lo = __builtin_elementwise_min(a, b), hi = __builtin_elementwise_max(a, b);
  return up ? hi : lo;
}
template <int M, int R>
__device__ __forceinline__ void pk_lanes_reverse_pair(short2_t (&v)[R], bool up) {
#pragma unroll
  for (int i = 0; i < R / 2; ++i) {
    const short2_t a = xor_mov<M>(v[R - 1 - i]);
    const short2_t b = xor_mov<M>(v[i]);
    v[i] = pk_pick(v[i], a, up);
    v[R - 1 - i] = pk_pick(v[R - 1 - i], b, up);
  }
}
template <int M, int R>
__device__ __forceinline__ void pk_lanes_cross_stage(short2_t (&v)[R], int sub) {
  const bool up = (sub & M) != 0;
#pragma unroll
  for (int i = 0; i < R; ++i) v[i] = pk_pick(v[i], xor_mov<M>(v[i]), up);
}
template <int R>
__device__ __forceinline__ void pk_lane_bitonic_merge(short2_t (&v)[R]) {
#pragma unroll
  for (int d = R / 2; d > 0; d /= 2) {
#pragma unroll
    for (int i = 0; i < R; ++i)
      if ((i & d) == 0) cmpx(v[i], v[i + d]);
  }
}
template <int G, int P, int R>
__device__ __forceinline__ void pk_lanes_merge_levels(short2_t (&v)[R], int sub) {
  if constexpr (G < P) {
    static_assert(G <= 16, "lane groups of at most 32");
    pk_lanes_reverse_pair<G - 1>(v, (sub & (G / 2)) != 0);
    if constexpr (G == 16) pk_lanes_cross_stage<4>(v, sub);
    if constexpr (G >= 8) pk_lanes_cross_stage<2>(v, sub);
    if constexpr (G >= 4) pk_lanes_cross_stage<1>(v, sub);
    pk_lane_bitonic_merge(v);
    pk_lanes_merge_levels<G * 2, P, R>(v, sub);
  }
}

// packed ±inf pair in each 16-bit element type: a padded slot's 32-bit load
template <class E>
__device__ uint32_t g_median_pad2[2] = {E::kNegInf * 0x10001u, E::kPosInf * 0x10001u};

// ---------------------------------------------------------------------------
// 16-bit order keys: x ^ 0x8000 for a non-negative value, ~x for a negative
// one, so that integer order is float order (-0 < +0; NaN above +inf or below
// -inf, a NaN column's result is replaced by its first NaN anyway); the
// inverse on a packed pair:
__device__ __forceinline__ uint32_t pk16_from_ukey(uint32_t k) {
  const uint32_t s = __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2_t, k) >> short(15));  // 0xffff: positive
  return k ^ (~s | 0x80008000u);
}
// sum of x over the P adjacent lanes of a column group (every lane gets it)
template <int P>
__device__ __forceinline__ int lanes_sum(int x) {
  if constexpr (P >= 2) x += __builtin_amdgcn_update_dpp(0, x, dpp_xor_ctrl<1>(), 0xf, 0xf, false);
  if constexpr (P >= 4) x += __builtin_amdgcn_update_dpp(0, x, dpp_xor_ctrl<2>(), 0xf, 0xf, false);
  if constexpr (P >= 8) x += __builtin_amdgcn_update_dpp(0, x, 0x141, 0xf, 0xf, false);  // row_half_mirror: quads
  if constexpr (P >= 16) x += __builtin_amdgcn_update_dpp(0, x, 0x140, 0xf, 0xf, false);  // row_mirror: halves
  if constexpr (P >= 32) x += __shfl_xor(x, 16, 64);
  return x;
}
// ---------------------------------------------------------------------------
// Selection on bit planes.  Counting with v_sad_u8 (rounds 4-5) cost two
// instructions per 4 keys per bit; on bit planes a 32-bit register holds one
// bit of 32 keys, so a most-significant-first radix select costs 4
// instructions per 32 keys per bit (and, popcount, xor, select):
//   - the lane's R packed words (client j's key pair: column 0 low, column 1
//     high) are transposed IN PLACE into planes: word j = 32 g + i holds bit
//     16 c + b of client 32 g + i's pair; five swap stages exchange register
//     index bit k with position bit k (i4 <-> c at 16, i3 <-> b3 at 8, whole
//     bytes: one v_perm_b32 per word; i2, i1, i0 <-> b2, b1, b0 at 4, 2, 1:
//     a shift and a v_bfi_b32 per word), after which word 32 g + 16 c + b is
//     plane b of column c for clients 32 g .. 32 g + 31;
//   - the float -> unsigned order key map (~x for a negative x, x | 0x8000
//     otherwise) is an xor of every plane with the sign plane, folded into
//     storing the COMPLEMENTED key planes Z_b (a 1 where the key's bit b is 0);
//   - per bit, most significant first, per column: c0 = #(active keys whose
//     bit is 0) summed over the column's P lanes (DPP); the median (rank
//     KMAX/2 - 1, the padding's fixed slot) has bit 0 if rank < c0 (active &=
//     Z_b), else bit 1 (rank -= c0, active &= ~Z_b).
// Per lane at K = 512 (two columns of 128 clients): 1,024 transpose, 128
// key-map and ~700 select instructions for 256 keys, where the byte-wise
// counting took ~3,600 (2,048 v_sad_u8; NOTES.md §5b).
template <int S, int D, int R>
__device__ __forceinline__ void slice_swap_stage(uint32_t (&w)[R]) {
#pragma unroll
  for (int j = 0; j < R; ++j) {
    if (j & D) continue;
    const uint32_t a = w[j], b = w[j + D];
    if constexpr (S == 16) {
      w[j] = __builtin_amdgcn_perm(b, a, 0x05040100u);      // {a.lo, b.lo}
      w[j + D] = __builtin_amdgcn_perm(b, a, 0x07060302u);  // {a.hi, b.hi}
    } else if constexpr (S == 8) {
      w[j] = __builtin_amdgcn_perm(b, a, 0x06020400u);      // {a0, b0, a2, b2}
      w[j + D] = __builtin_amdgcn_perm(b, a, 0x07030501u);  // {a1, b1, a3, b3}
    } else {
      constexpr uint32_t m = S == 4 ? 0x0f0f0f0fu : S == 2 ? 0x33333333u : 0x55555555u;
      w[j] = (a & m) | ((b << S) & ~m);
      w[j + D] = ((a >> S) & m) | (b & ~m);
    }
  }
}
// words 32 g .. 32 g + 31 of w: raw key pairs -> complemented order-key planes
template <int R>
__device__ __forceinline__ void pk16_slice_planes_group(uint32_t (&w)[R], int g) {
  uint32_t (&v)[32] = *reinterpret_cast<uint32_t (*)[32]>(&w[32 * g]);
  slice_swap_stage<16, 16, 32>(v);
  slice_swap_stage<8, 8, 32>(v);
  slice_swap_stage<4, 4, 32>(v);
  slice_swap_stage<2, 2, 32>(v);
  slice_swap_stage<1, 1, 32>(v);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const uint32_t ns = ~v[16 * c + 15];  // 1: a non-negative value
#pragma unroll
    for (int b = 0; b < 15; ++b) v[16 * c + b] ^= ns;
    // Z_15 = the sign plane itself
  }
}
// the radix select over the planes of pk16_slice_planes_group
template <int P, int R>
__device__ __forceinline__ uint32_t pk16_slice_select(const uint32_t (&w)[R]) {
  constexpr int G = R / 32;
  uint32_t act[2][G];
  uint32_t key[2] = {0u, 0u};
  int rank[2] = {P * R / 2 - 1, P * R / 2 - 1};
#pragma unroll
  for (int b = 15; b >= 0; --b) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      uint32_t t[G];
      uint32_t n = 0;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const uint32_t z = w[32 * g + 16 * c + b];
        t[g] = b == 15 ? z : (act[c][g] & z);
        n = __builtin_popcount(t[g]) + n;
      }
      const int c0 = lanes_sum<P>(int(n));
      const bool one = c0 <= rank[c];
      rank[c] -= one ? c0 : 0;
      key[c] = 2u * key[c] + (one ? 1u : 0u);
      if (b > 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const uint32_t a = b == 15 ? ~0u : act[c][g];
          act[c][g] = one ? (a ^ t[g]) : t[g];
        }
      }
    }
  }
  return key[0] | (key[1] << 16);
}

// PLANES: the median by the bit-plane radix select, planes built group by
// group as the loads land (a wave holding a NaN re-reads its words for the
// first NaN); otherwise by the sorting networks and cross-lane merges
template <int P, int R, bool FULL, bool TAIL, class E, int BS = 256, bool PLANES = false>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(2))) void median_pk16_lanes_kernel(
    const uint16_t* const* __restrict__ src, int K, int64_t pairs, uint16_t* __restrict__ out, int64_t pair0) {
  static_assert((PLANES && P == 1) || P == 2 || P == 4 || P == 8 || P == 16 || P == 32,
                "2 to 32 lanes per column pair (1 for the bit-plane select)");
  static_assert(R == 32 || R == 64 || R == 128, "32, 64 or 128 values per lane");
  constexpr int KMAX = P * R, PAD = 2;
  __shared__ const uint16_t* rows[KMAX + PAD * P];
  __shared__ uint64_t offmask[FULL ? 1 : KMAX + PAD * P];
  const int t = threadIdx.x, sub = t & (P - 1);
  if constexpr (FULL) K = KMAX;
  const int below = KMAX / 2 - 1 - (K - 1) / 2;  // -inf pads; the rest of the padding is +inf
  for (int i = t; i < KMAX; i += BS) {
    const int q = i + PAD * (i / R);
    if (FULL || i < K) {
      rows[q] = src[i];
      if constexpr (!FULL) offmask[q] = ~uint64_t(0);
    } else {
      rows[q] = reinterpret_cast<const uint16_t*>(&g_median_pad2<E>[i - K < below ? 0 : 1]);
      offmask[q] = 0;
    }
  }
  __syncthreads();
  // TAIL: `pairs` is the index of the pair holding the lone last column.
  // Otherwise a column group past the end recomputes the last pair and does
  // not store (every lane stays active through the DPP exchanges).
  const int64_t e = TAIL ? pairs : pair0 + (int64_t(blockIdx.x) * BS + t) / P;
  const uint64_t boff = uint64_t(TAIL || e < pairs ? e : pairs - 1) * 4u;
  auto word = [&](int j) -> uint32_t {
    const int q = sub * (R + PAD) + j;
    const uint64_t off = FULL ? boff : (boff & offmask[q]);
    const auto row = reinterpret_cast<const char*>(rows[q]);
    if constexpr (TAIL)
      return uint32_t(*as_global(reinterpret_cast<const uint16_t*>(row + off))) * 0x10001u;
    else
      return lanes_load(as_global(reinterpret_cast<const uint32_t*>(row + off)));
  };
  uint32_t raw[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    if (j % 16 == 0 && j) __builtin_amdgcn_sched_barrier(0);
    raw[j] = word(j);
  }
  __builtin_amdgcn_sched_barrier(0);  // every load in flight before the first test
  uint32_t nanacc = 0;  // per half, max of |x| bits
  auto nan_max = [&](uint32_t x) {
    nanacc = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(ushort2_t, nanacc),
                                                                    __builtin_bit_cast(ushort2_t, x & 0x7fff7fffu)));
  };
  if constexpr (PLANES) {
    // planes group by group as the group's loads land (the swap stages pair
    // words inside a 32-word group): the raw words are gone afterwards, so a
    // wave holding a NaN reloads them below
#pragma unroll
    for (int g = 0; g < R / 32; ++g) {
#pragma unroll
      for (int j = 32 * g; j < 32 * g + 32; ++j) nan_max(raw[j]);
      pk16_slice_planes_group<R>(raw, g);
    }
  } else {
#pragma unroll
    for (int j = 0; j < R; ++j) nan_max(raw[j]);
  }
  // first NaN per half in client (= slot) order as (slot << 16 | bits), only
  // in waves holding a NaN column; KMAX << 16: none
  int first_lo = KMAX << 16, first_hi = KMAX << 16;
  if (__ballot((nanacc & 0xffffu) > E::kPosInf || (nanacc >> 16) > E::kPosInf)) {
#pragma unroll
    for (int j = R - 1; j >= 0; --j) {  // predicated, walked backwards: the lowest slot wins
      const uint32_t x = PLANES ? word(j) : raw[j];
      const int s = (sub * R + j) << 16;
      if ((x & 0x7fffu) > E::kPosInf) first_lo = s | int(x & 0xffffu);
      if (((x >> 16) & 0x7fffu) > E::kPosInf) first_hi = s | int(x >> 16);
    }
#pragma unroll
    for (int m = 1; m < P; m <<= 1) {
      first_lo = min(first_lo, __shfl_xor(first_lo, m, 64));
      first_hi = min(first_hi, __shfl_xor(first_hi, m, 64));
    }
  }
  uint32_t bits;
  if constexpr (PLANES) {
    bits = pk16_from_ukey(pk16_slice_select<P, R>(raw));
  } else {
  short2_t v[R];
#pragma unroll
  for (int j = 0; j < R; ++j) v[j] = pk16_key(raw[j]);
  short2_t m;
  if constexpr (P == 4 && !kPk16Mirror) {
    // odd lanes hold complemented keys (~k reverses the int16 order): every
    // cross-lane step is min(own, ~partner) in every lane (lanes4_merge_median)
    const short2_t flip = (sub & 1) ? short2_t(short(-1)) : short2_t(short(0));
#pragma unroll
    for (int j = 0; j < R; ++j) v[j] ^= flip;
    pairwise_sort<R>(v);
    m = lanes4_merge_median(v);
  } else {
    pairwise_sort<R>(v);
    pk_lanes_merge_levels<2, P, R>(v, sub);
    // last level: the lower P/2 lanes keep the KMAX/2 smallest keys per half
    pk_lanes_reverse_pair<P - 1>(v, (sub & (P / 2)) != 0);
    m = v[0];
#pragma unroll
    for (int i = 1; i < R; ++i) m = __builtin_elementwise_max(m, v[i]);
    if constexpr (P >= 4) m = __builtin_elementwise_max(m, dpp_mov<dpp_xor_ctrl<1>()>(m));
    if constexpr (P >= 8) m = __builtin_elementwise_max(m, dpp_mov<dpp_xor_ctrl<2>()>(m));
    if constexpr (P >= 16) m = __builtin_elementwise_max(m, dpp_mov<dpp_xor_ctrl<7>()>(m));  // quad maxima
    if constexpr (P >= 32) m = __builtin_elementwise_max(m, dpp_mov<dpp_xor_ctrl<15>()>(m));  // row halves
  }
  bits = pk16_bits(m);
  }
  if (first_lo < (KMAX << 16)) bits = (bits & 0xffff0000u) | (uint32_t(first_lo) & 0xffffu);
  if (first_hi < (KMAX << 16)) bits = (bits & 0xffffu) | (uint32_t(first_hi) << 16);
  if constexpr (TAIL) {
    if (t == 0) out[2 * e] = uint16_t(bits);
  } else if (sub == 0 && e < pairs) {
    *reinterpret_cast<uint32_t*>(out + 2 * e) = bits;
  }
}

template <int P, int R, class E, int BS = 256, bool PLANES = false>
int launch_median_pk16_lanes(const uint16_t* const* src, int K, int64_t N, uint16_t* out, hipStream_t st,
                             int64_t pair0 = 0) {
  const int64_t pairs = N / 2;
  const int64_t grid = ((pairs - pair0) * P + BS - 1) / BS;
  if (grid > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, "fedagg_median: N too large");
  if (pairs > pair0) {
    if (K == P * R)
      hipLaunchKernelGGL((median_pk16_lanes_kernel<P, R, true, false, E, BS, PLANES>), dim3(unsigned(grid)),
                         dim3(BS), 0, st, src, K, pairs, out, pair0);
    else
      hipLaunchKernelGGL((median_pk16_lanes_kernel<P, R, false, false, E, BS, PLANES>), dim3(unsigned(grid)),
                         dim3(BS), 0, st, src, K, pairs, out, pair0);
  }
  if (N & 1)
    hipLaunchKernelGGL((median_pk16_lanes_kernel<P, R, false, true, E, BS, PLANES>), dim3(1), dim3(BS), 0, st, src,
                       K, pairs, out, int64_t(0));
  return check_launch("fedagg_median");
}

// ---------------------------------------------------------------------------
// Streamed form of the bit-plane selection (128 < K <= 1024, 16-bit rows).
// The register kernel above loads a wave's 32 KB, then selects: its waves
// convoy (they start together, share the SIMD while selecting, and all wait
// for memory again together), so it runs near the SUM of its memory time and
// its selection time.  Here persistent blocks stage the NEXT column block in
// LDS by LDS-DMA (global_load_lds_dwordx4, no registers) while their waves
// select the current one:
//   - each block walks a contiguous range of column blocks (its own share of
//     every row, read front to back: the loads ran at 0.80 of HBM this way
//     against 0.69 with a grid stride, whose blocks all work in the same
//     64-KB window of every row);
//   - the tile's DMA instructions read whole 128-B lines of the rows,
//     non-temporal (every byte is read once: 0.80 against 0.74 of HBM for
//     the loads alone, NOTES.md §5b); rows at or above K read a 16-B pad of
//     -inf / +inf (the register kernel's padding, so the median stays at rank
//     KMAX / 2 - 1);
//   - a row's 16-B chunks are stored XOR-swizzled so that the 64 lanes of a
//     ds_read hit 64 banks; the DMA applies the inverse permutation to its
//     SOURCE chunks (its LDS side is lane-linear);
//   - per column block: wait for the own DMA, barrier, read the lane's
//     words, barrier, issue the own share of the next column block's DMA into
//     the same tile, then the planes, the radix select and the store.
// The columns past the last whole column block (and the odd last column) run
// through median_pk16_lanes_kernel with a pair offset.
template <class E>
__device__ __attribute__((aligned(16))) uint32_t g_median_pad16[2][4] = {
    {E::kNegInf * 0x10001u, E::kNegInf * 0x10001u, E::kNegInf * 0x10001u, E::kNegInf * 0x10001u},
    {E::kPosInf * 0x10001u, E::kPosInf * 0x10001u, E::kPosInf * 0x10001u, E::kPosInf * 0x10001u}};

// A wave's share of a streamed tile's LDS-DMA: NK instructions of 64 lanes x
// 16 B (1 KB each, instruction k at LDS base + WAVES k KB: the block's waves
// interleave), non-temporal.  The per-lane source pointers live in registers
// and step one column block per next(); pad rows do not step.
template <int NK, int WAVES = 4>
struct TileDma {
  const char* src[NK];
  uint32_t step[NK];
  __device__ __forceinline__ void issue(unsigned char* lds) const {
#pragma unroll
    for (int k = 0; k < NK; ++k)
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(src[k]),
                                       (void __attribute__((address_space(3)))*)(lds + k * WAVES * 1024), 16, 0, 2);
  }
  __device__ __forceinline__ void next() {
#pragma unroll
    for (int k = 0; k < NK; ++k) src[k] += step[k];
  }
};

// this block's contiguous range [b, b_end) of the nblk column blocks
__device__ __forceinline__ void block_range(int64_t nblk, int64_t& b, int64_t& b_end) {
  const int64_t per = (nblk + gridDim.x - 1) / gridDim.x;
  b = int64_t(blockIdx.x) * per;
  b_end = b + per < nblk ? b + per : nblk;
}

// ---------------------------------------------------------------------------
// One column per lane.  The register kernel above gives a lane two columns
// of R clients and spends a v_perm_b32 per word separating the columns (swap
// stage 16) and, per bit, the P-lane count reduction for two columns (a
// streamed form of it, measured in round 6, ran config 4 in 16.7 ms against
// 15.0-15.6 for this one).  Here a lane's word j holds ONE column of two
// clients, 2 (P j + s) in the low half and the next client in the high half,
// assembled from the LDS tile by two 16-bit reads and a v_perm_b32; the half
// bit is a client bit, so four swap
// stages (8, 4, 2, 1) on groups of 16 words make the planes: word 16 g + b is
// plane b of clients 32 g .. 32 g + 31 of the lane (the lane's client
// 2 (P (16 g + i) + s) + h at position 2 i + h).  A lane holds 2 R clients of
// its column, P = KMAX / (2 R) lanes per column.
//   - Block: WAVES waves x 64 / P columns = WAVES * 128 / P bytes of every
//     row per column block (one 128-B line for (P, WAVES) = (4, 4) and
//     (8, 8)); tile KMAX x that, R DMA instructions per wave-quarter; up to
//     512 clients (4, 64, 4): 2 blocks per CU; up to 1024 (8, 64, 8): one
//     block of 8 waves per CU (K = 1024 over 4M columns 1.43 ms against 1.85
//     for the streamed pair form; profiles/r06/q/).
//   - Per lane at K = 512: ~900 VALU instructions for its 128 keys (the pair
//     form: ~1,500); config 4's median 15.0 ms against 16.7 ms for the pair
//     form and 21.7 ms for the byte-wise counting (NOTES.md §5b).
//   - Chunk swizzle: row r's 16-B chunk c is stored at c ^ ((8 / P) * ((r / 2)
//     % P)), so the P row pairs one read covers land in different banks.
//   - NaN: found on the raw planes (all exponent planes set and a mantissa
//     plane set); a wave holding one re-reads its columns from memory for the
//     first NaN in client order (the tile is being refilled by then).
template <int P>
__device__ __forceinline__ constexpr int colswz(int r) {
  return (8 / P) * ((r / 2) % P);
}

// blocks of the column kernel that fit a CU's 160 KB of LDS
template <int P, int R, int WAVES>
constexpr int colstream_blocks_per_cu() {
  return 163840 / (2 * P * R * WAVES * 128 / P + 2 * P * R * 8);
}
template <int P, int R, int WAVES, bool FULL, class E>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(
    colstream_blocks_per_cu<P, R, WAVES>() * WAVES / 4))) void
median_pk16_colstream_kernel(const uint16_t* const* __restrict__ src, int K, int64_t nblk,
                             uint16_t* __restrict__ out) {
  static_assert(P == 2 || P == 4 || P == 8, "2, 4 or 8 lanes per column");
  static_assert(R == 32 || R == 64, "32 or 64 words (64 or 128 clients) per lane");
  constexpr int KMAX = 2 * P * R, WB = 128 / P;  // tile rows, a wave's bytes of a tile row
  constexpr int RB = WAVES * WB;                 // bytes per tile row (the column block's bytes)
  constexpr int NC = RB / 16;                    // 16-B chunks per tile row = DMA lanes per row
  constexpr int TILE = KMAX * RB;                // R * WAVES / 4 KB
  static_assert(8 * (P - 1) / P < NC, "the chunk swizzle stays inside a row");
  __shared__ __attribute__((aligned(16))) unsigned char smem[TILE + KMAX * 8];
  auto rows = reinterpret_cast<const char**>(smem + TILE);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if constexpr (FULL) K = KMAX;
  const int below = KMAX / 2 - 1 - (K - 1) / 2;  // -inf pads; the rest of the padding is +inf
  for (int i = t; i < KMAX; i += 64 * WAVES)
    rows[i] = (FULL || i < K) ? reinterpret_cast<const char*>(src[i])
                              : reinterpret_cast<const char*>(g_median_pad16<E>[i - K < below ? 0 : 1]);
  __syncthreads();
  int64_t b, b_end;
  block_range(nblk, b, b_end);
  // DMA share of this wave: instructions i = WAVES k + wave, lane -> tile row
  // (1024 / RB) i + lane / NC, stored chunk lane % NC = source chunk ^ swz(row)
  unsigned char* const tile_w = smem + __builtin_amdgcn_readfirstlane(wave) * 1024;
  TileDma<R / 4, WAVES> dma;
#pragma unroll
  for (int k = 0; k < R / 4; ++k) {
    const int r = (1024 / RB) * (WAVES * k + wave) + lane / NC;
    const int c = (lane % NC) ^ colswz<P>(r);
    const bool real = FULL || r < K;
    dma.src[k] = real ? rows[r] + (uint64_t(b) * RB + uint64_t(c) * 16u) : rows[r];
    dma.step[k] = real ? uint32_t(RB) : 0u;
  }
  const int sub = lane & (P - 1), p = lane / P;
  // word j: rows 2 (P j + sub) and + 1, column byte cb = wave * WB + 2 p,
  // chunk cb / 16 stored at ^ swz (the same for both rows and every j)
  const int cb = wave * WB + 2 * p;
  const int pos = (cb / 16) ^ colswz<P>(2 * sub);
  const uint16_t* tlo = reinterpret_cast<const uint16_t*>(smem + 2 * sub * RB + pos * 16 + (cb & 15));
  constexpr int JS = P * RB;  // 16-bit elements between words j and j + 1 (2 P rows)
  if (b < b_end) dma.issue(tile_w);
  for (; b < b_end; ++b) {
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): this wave's DMA has landed
    __builtin_amdgcn_s_barrier();        // ... and every wave's
    __builtin_amdgcn_sched_barrier(0);
    // each word from two 16-bit reads (gfx950's d16 reads, which would merge
    // the halves in the register file, zero the other half under SRAM ECC:
    // hipcc merges them with a v_perm_b32 per word)
    uint32_t w[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      ushort2_t v;
      v.x = tlo[j * JS];
      v.y = tlo[j * JS + RB / 2];
      w[j] = __builtin_bit_cast(uint32_t, v);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): every word read ...
    __builtin_amdgcn_s_barrier();        // ... by every wave before the tile is refilled
    __builtin_amdgcn_sched_barrier(0);
    const int64_t bcur = b;
    if (b + 1 < b_end) {
      dma.next();
      dma.issue(tile_w);
    }
    // planes: four swap stages per 16-word group
    constexpr int MB = __builtin_ctz(E::kPosInf);  // mantissa bits
    uint32_t nan = 0;
#pragma unroll
    for (int g = 0; g < R / 16; ++g) {
      uint32_t (&v)[16] = *reinterpret_cast<uint32_t (*)[16]>(&w[16 * g]);
      slice_swap_stage<8, 8, 16>(v);
      slice_swap_stage<4, 4, 16>(v);
      slice_swap_stage<2, 2, 16>(v);
      slice_swap_stage<1, 1, 16>(v);
      uint32_t e = v[14], m = v[0];
#pragma unroll
      for (int q = MB; q < 14; ++q) e &= v[q];
#pragma unroll
      for (int q = 1; q < MB; ++q) m |= v[q];
      nan |= e & m;
      const uint32_t ns = ~v[15];  // 1: a non-negative value
#pragma unroll
      for (int q = 0; q < 15; ++q) v[q] ^= ns;  // complemented order-key planes; Z_15 = the sign plane
    }
    // the select: rank KMAX / 2 - 1 over the column's P lanes
    constexpr int G = R / 16;
    uint32_t act[G];
    uint32_t key = 0;
    int rank = KMAX / 2 - 1;
#pragma unroll
    for (int q = 15; q >= 0; --q) {
      uint32_t tq[G];
      uint32_t n = 0;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const uint32_t z = w[16 * g + q];
        tq[g] = q == 15 ? z : (act[g] & z);
        n = __builtin_popcount(tq[g]) + n;
      }
      const int c0 = lanes_sum<P>(int(n));
      const bool one = c0 <= rank;
      rank -= one ? c0 : 0;
      key = 2u * key + (one ? 1u : 0u);
      if (q > 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const uint32_t a = q == 15 ? ~0u : act[g];
          act[g] = one ? (a ^ tq[g]) : tq[g];
        }
      }
    }
    // order key -> bits (the 16-bit form of pk16_from_ukey)
    uint32_t bits = (key & 0x8000u) ? (key ^ 0x8000u) : (~key & 0xffffu);
    if (__ballot(nan != 0)) {
      // first NaN of the column in client order, from memory
      int first = KMAX;
      uint32_t fb = 0;
      const uint64_t off = uint64_t(bcur) * RB + uint64_t(cb);
      for (int j = R - 1; j >= 0; --j) {
#pragma unroll
        for (int h = 1; h >= 0; --h) {
          const int r = 2 * (P * j + sub) + h;
          if (r < K) {
            const uint32_t x = *as_global(reinterpret_cast<const uint16_t*>(rows[r] + off));
            if ((x & 0x7fffu) > E::kPosInf) {
              first = r;
              fb = x;
            }
          }
        }
      }
#pragma unroll
      for (int m2 = 1; m2 < P; m2 <<= 1) {
        const int of = __shfl_xor(first, m2, 64);
        const uint32_t ob = __shfl_xor(fb, m2, 64);
        if (of < first) {
          first = of;
          fb = ob;
        }
      }
      if (first < KMAX) bits = fb;
    }
    if (sub == 0) out[bcur * (RB / 2) + wave * (64 / P) + p] = uint16_t(bits);
  }
}

// CUs of the current device (the persistent kernels' resident grid), cached
// per device; callers on several threads may race to fill an entry with the
// same value, hence the relaxed atomics
int device_cu_count() {
  static std::atomic<int> cus[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int n = cus[dev].load(std::memory_order_relaxed);
  if (n <= 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

template <int P, int R, int WAVES, class E>
int launch_median_pk16_colstream(const uint16_t* const* src, int K, int64_t N, uint16_t* out, hipStream_t st) {
  constexpr int COLS = WAVES * 64 / P;  // columns per column block
  const int64_t nblk = N / COLS;
  if (nblk > 0) {
    const int64_t cap = int64_t(device_cu_count()) * colstream_blocks_per_cu<P, R, WAVES>();  // resident
    const int64_t grid = nblk < cap ? nblk : cap;
    if (K == 2 * P * R)
      hipLaunchKernelGGL((median_pk16_colstream_kernel<P, R, WAVES, true, E>), dim3(unsigned(grid)),
                         dim3(64 * WAVES), 0, st, src, K, nblk, out);
    else
      hipLaunchKernelGGL((median_pk16_colstream_kernel<P, R, WAVES, false, E>), dim3(unsigned(grid)),
                         dim3(64 * WAVES), 0, st, src, K, nblk, out);
    if (int rc = check_launch("fedagg_median")) return rc;
  }
  // the remaining columns (fewer than one column block) and the odd last one
  return launch_median_pk16_lanes<2 * P * R / 128, 128, E, 256, true>(src, K, N, out, st, nblk * (COLS / 2));
}

// Any number of clients (the path above 1024, where the lane-group sort runs
// out of lanes per column): MSD radix select over 32-bit order keys, the
// column tile streamed from memory once per 8-bit digit.  A block owns 64
// consecutive columns; its 4 waves read rows q, q + 4, ... of all 64 (one
// coalesced 64-column segment per wave instruction) and count the keys that
// match the digits chosen so far into a per-column 256-bin LDS histogram;
// then, per column, the bin holding the remaining rank gives the next digit.
// Four passes fix all 32 bits.  Passes 2-4 re-read the tile (K x 256 B per
// row group), mostly from L2 / MALL.  The NaN rule is the register kernels':
// the column's first NaN in client order (an LDS atomic min on the row, pass
// one).  Exact for every input; a ±0 tie at the median may return the other
// zero than torch's nth_element, as everywhere.
constexpr int kRsCols = 64;
__device__ __forceinline__ uint32_t f32_order_key(uint32_t u) { return (u & 0x80000000u) ? ~u : (u | 0x80000000u); }
__device__ __forceinline__ uint32_t f32_from_order_key(uint32_t k) { return (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k; }

template <class E>
__global__ __launch_bounds__(256) void median_radix_stream_kernel(const typename E::S* const* __restrict__ src, int K,
                                                                  int64_t N, typename E::S* __restrict__ out) {
  constexpr int HS = 257;  // bins per column + 1: column c starts c banks apart
  __shared__ uint32_t hist[kRsCols * HS];
  __shared__ uint32_t part[4][kRsCols];
  __shared__ uint32_t s_prefix[kRsCols];
  __shared__ int s_rank[kRsCols];
  __shared__ int nan_row[kRsCols];
  const int t = threadIdx.x, c = t & (kRsCols - 1), q = t >> 6;
  const int64_t col = int64_t(blockIdx.x) * kRsCols + c;
  const int64_t colc = col < N ? col : N - 1;  // columns past the end recompute the last one
  if (q == 0) {
    nan_row[c] = K;
    s_prefix[c] = 0;
    s_rank[c] = (K - 1) / 2;
  }
  uint32_t pmask = 0;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = t; i < kRsCols * HS; i += 256) hist[i] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix[c];
    int first_nan = K;
    int r = q;
    for (; r + 12 < K; r += 16) {  // 4 rows in flight per lane
      typename E::S x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = __builtin_nontemporal_load(as_global(src[r + 4 * u]) + colc);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float v = E::widen(x[u]);
        const uint32_t k = f32_order_key(__float_as_uint(v));
        if (shift == 24 && E::raw_nan(x[u]) && first_nan == K) first_nan = r + 4 * u;
        if ((k & pmask) == prefix) atomicAdd(&hist[c * HS + ((k >> shift) & 0xffu)], 1u);
      }
    }
    for (; r < K; r += 4) {
      const typename E::S x = __builtin_nontemporal_load(as_global(src[r]) + colc);
      const uint32_t k = f32_order_key(__float_as_uint(E::widen(x)));
      if (shift == 24 && E::raw_nan(x) && first_nan == K) first_nan = r;
      if ((k & pmask) == prefix) atomicAdd(&hist[c * HS + ((k >> shift) & 0xffu)], 1u);
    }
    if (first_nan < K) atomicMin(&nan_row[c], first_nan);
    __syncthreads();
    // lane (c, q) owns bins [64q, 64q + 64) of column c
    uint32_t own = 0;
    for (int b = 0; b < 64; ++b) own += hist[c * HS + 64 * q + b];
    part[q][c] = own;
    __syncthreads();
    const int rank = s_rank[c];
    int below = 0;
    for (int j = 0; j < q; ++j) below += int(part[j][c]);
    if (below <= rank && rank < below + int(own)) {  // exactly one q per column
      int b = 0;
      for (; b < 63; ++b) {
        const int h = int(hist[c * HS + 64 * q + b]);
        if (below + h > rank) break;
        below += h;
      }
      s_prefix[c] = prefix | (uint32_t(64 * q + b) << shift);
      s_rank[c] = rank - below;
    }
    pmask |= 0xffu << shift;
    __syncthreads();
  }
  if (q == 0 && col < N) {
    const int nr = nan_row[c];
    out[col] = nr < K ? as_global(src[nr])[col] : E::narrow(__uint_as_float(f32_from_order_key(s_prefix[c])));
  }
}

template <class E>
int launch_median_radix_stream(const typename E::S* const* src, int K, int64_t N, typename E::S* out, hipStream_t st) {
  const int64_t grid = (N + kRsCols - 1) / kRsCols;
  if (grid > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, "fedagg_median: N too large");
  hipLaunchKernelGGL((median_radix_stream_kernel<E>), dim3(unsigned(grid)), dim3(256), 0, st, src, K, N, out);
  return check_launch("fedagg_median");
}


template <class E>
int median_dispatch(const typename E::S* const* d_src, int32_t K, int64_t N, typename E::S* d_out, bool aligned,
                    hipStream_t st) {
  if (K > 128) {  // 4 or 8 lanes per column, register sorts + cross-lane merges
    if constexpr (sizeof(typename E::S) == 2) {
      if (aligned && K <= 4096) {  // two columns per lane on packed int16 keys
        // the bit-plane radix select streamed through LDS, one column per lane
        if (K <= 256) return launch_median_pk16_colstream<2, 64, 4, E>(d_src, K, N, d_out, st);
        if (K <= 512) return launch_median_pk16_colstream<4, 64, 4, E>(d_src, K, N, d_out, st);
        if (K <= 1024) return launch_median_pk16_colstream<8, 64, 8, E>(d_src, K, N, d_out, st);
        if (K <= 2048) return launch_median_pk16_lanes<16, 128, E>(d_src, K, N, d_out, st);
        return launch_median_pk16_lanes<32, 128, E>(d_src, K, N, d_out, st);
      }
    }
    if (K <= 256) return launch_median_lanes<4, 64, E>(d_src, K, N, d_out, st);  // 1.1 ms vs 1.4 for <2, 128> (4M cols)
    if (K <= 512) return launch_median_lanes<4, 128, E>(d_src, K, N, d_out, st);
    if (K <= 1024) return launch_median_lanes<8, 128, E>(d_src, K, N, d_out, st);
    if (K <= 2048) return launch_median_lanes<16, 128, E>(d_src, K, N, d_out, st);
    // 32 lanes per column pay off against the radix select only well inside
    // their range (1M columns: 18.9 vs 18.7 ms at K = 2,049, 22.9 vs 35.4 ms
    // at 4,096 in fp32; the packed 16-bit kernels win at every K, above)
    if (K > 2560 && K <= 4096) return launch_median_lanes<32, 128, E>(d_src, K, N, d_out, st);
    return launch_median_radix_stream<E>(d_src, K, N, d_out, st);  // no bound on K
  }
  if constexpr (sizeof(typename E::S) == 2) {
    if (aligned) {  // two columns per lane on packed int16 keys
      if (K <= 32) return launch_median_pk16<32, E>(d_src, K, N, d_out, st);
      if (K <= 64) return launch_median_pk16<64, E>(d_src, K, N, d_out, st);
      if (K <= 96) return launch_median_pk16<96, E>(d_src, K, N, d_out, st);
      // 97..128: the bit-plane select, one lane per column pair holding all
      // 128 slots (the 128-slot network padded K = 100 to 0.42 ms per 8M
      // columns against 0.33; 3.79 vs 3.70 ms at config 4's 128 clients;
      // below 97 the networks' smaller tiers win: NOTES.md §5b, round 6)
      return launch_median_pk16_lanes<1, 128, E, 256, true>(d_src, K, N, d_out, st);
    }
  }
  if (K <= 8) return launch_median<8, E>(d_src, K, N, d_out, st);
  if (K <= 16) return launch_median<16, E>(d_src, K, N, d_out, st);
  if (K <= 24) return launch_median<24, E>(d_src, K, N, d_out, st);
  if (K <= 32) return launch_median<32, E>(d_src, K, N, d_out, st);
  if (K <= 48) return launch_median<48, E>(d_src, K, N, d_out, st);
  if (K <= 64) return launch_median<64, E>(d_src, K, N, d_out, st);
  if (K <= 96) return launch_median<96, E>(d_src, K, N, d_out, st);
  return launch_median<128, E>(d_src, K, N, d_out, st);
}


}  // namespace

extern "C" {

int fedagg_median(int32_t dtype, const void* const* d_src, int32_t K, int64_t N, void* d_out, uint32_t flags,
                  fedagg_stream_t stream) {
  const bool aligned = (flags & FEDAGG_ALIGNED16) != 0;
  if (K < 1 || N < 0) return set_error(FEDAGG_EINVAL, "fedagg_median: K must be >= 1 and N >= 0");
  if (!d_src || !d_out) return set_error(FEDAGG_EINVAL, "fedagg_median: null pointer");
  if (N == 0) return FEDAGG_OK;
  auto st = reinterpret_cast<hipStream_t>(stream);
  switch (dtype) {
    case FEDAGG_DT_F32:
      return median_dispatch<MedF32>(reinterpret_cast<const float* const*>(d_src), K, N,
                                     static_cast<float*>(d_out), aligned, st);
    case FEDAGG_DT_BF16:
      return median_dispatch<MedBF16>(reinterpret_cast<const uint16_t* const*>(d_src), K, N,
                                      static_cast<uint16_t*>(d_out), aligned, st);
    case FEDAGG_DT_F16:
      return median_dispatch<MedF16>(reinterpret_cast<const uint16_t* const*>(d_src), K, N,
                                     static_cast<uint16_t*>(d_out), aligned, st);
    default:
      return set_error(FEDAGG_EINVAL, "fedagg_median: dtype must be FEDAGG_DT_F32, _BF16 or _F16");
  }
}

int fedagg_median_f32(const float* const* d_src, int32_t K, int64_t N, float* d_out, uint32_t flags,
                      fedagg_stream_t stream) {
  return fedagg_median(FEDAGG_DT_F32, reinterpret_cast<const void* const*>(d_src), K, N, d_out, flags, stream);
}

}  // extern "C"
