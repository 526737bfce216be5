// Probe (tool only): radix selection with register-resident keys and per-column
// LDS histograms, for the coordinate-wise median above 128 clients.
//
// A column's K <= 4R values sit in the registers of 4 lanes (R each), as order
// keys.  Each 8-bit digit pass adds every key's digit into the column's
// 256-bin LDS histogram (one ds_add per value), finds the bin holding the
// target rank, and clamps every key into the bin's key range (a monotone map:
// the rank-k key is unchanged, no rank bookkeeping).  4 passes fix an fp32
// key.  The sorting-network kernels spend ~150 VALU cycles per value on
// half-rate min/max; this spends ~28 on mostly full-rate ops plus 4 LDS adds.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <class T>
__device__ __forceinline__ const T __attribute__((address_space(1)))* as_global(const T* p) {
  return (const T __attribute__((address_space(1)))*)(p);
}

__device__ float g_pad_f32[2] = {-__builtin_huge_valf(), __builtin_huge_valf()};

__device__ __forceinline__ uint32_t f32_key(uint32_t u) { return u ^ (uint32_t(int32_t(u) >> 31) | 0x80000000u); }
__device__ __forceinline__ uint32_t f32_from_key(uint32_t k) { return (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k; }

// (a & b) ^ c: the compiler emits one full-rate v_bitop3_b32 (plain C, so it
// picks the truth table; bitop3 indexes it as a*4 + b*2 + c)
__device__ __forceinline__ uint32_t and_xor(uint32_t a, uint32_t b, uint32_t c) { return (a & b) ^ c; }

// one v_med3_u32 (the compiler splits min(max()) into two half-rate ops when
// it cannot prove lo <= hi)
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t lo, uint32_t hi) {
  uint32_t d;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(lo), "v"(hi));
  return d;
}
// (a & b) | c as one full-rate v_bitop3_b32 (table index a*4 + b*2 + c: 0xEA)
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xea" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t lds_addr(const uint32_t* p) {
  return uint32_t(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) uint32_t*)(p)));
}
__device__ __forceinline__ void lds_add1(uint32_t a) {
  __hip_atomic_fetch_add((lds_u32*)(uintptr_t)(a), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int kCW = 16;    // columns per wave
constexpr int kBins = 256;

// Wave-private state: the 16 columns' histograms, the lanes' partial totals,
// the chosen prefix per column.
struct WaveLds {
  uint32_t part[kCW][4];
  uint32_t pfx[kCW];
  uint32_t flag[kCW];
};

template <int R, bool FULL>
__global__ __launch_bounds__(256) void median_rsel_f32_kernel(const float* const* __restrict__ src, int K, int64_t N,
                                                              float* __restrict__ out) {
  constexpr int P = 4, KMAX = P * R, PAD = 2;
  __shared__ __attribute__((aligned(1024))) uint32_t hist_all[4][kCW][kBins];  // 1 KB-aligned columns
  __shared__ WaveLds lds[4];
  __shared__ const float* rows[KMAX + PAD * P];
  __shared__ uint64_t offmask[FULL ? 1 : KMAX + PAD * P];
  const int t = threadIdx.x, w = t >> 6, l = t & 63, c = l & 15, sub = l >> 4;
  if constexpr (FULL) K = KMAX;
  const int below = KMAX / 2 - 1 - (K - 1) / 2;  // -inf pads; the rest of the padding is +inf
  for (int i = t; i < KMAX; i += 256) {
    const int q = i + PAD * (i / R);
    if (FULL || i < K) {
      rows[q] = src[i];
      if constexpr (!FULL) offmask[q] = ~uint64_t(0);
    } else {
      rows[q] = &g_pad_f32[i - K < below ? 0 : 1];
      offmask[q] = 0;
    }
  }
  WaveLds& L = lds[w];
  uint32_t (&hist)[kCW][kBins] = hist_all[w];
  // zero this wave's histograms: 16 x 256 words, 64 per lane
  {
    uint32_t* h = &hist[0][0];
#pragma unroll
    for (int i = 0; i < 16; ++i) *reinterpret_cast<u32x4*>(h + (i * 64 + l) * 4) = u32x4{0, 0, 0, 0};
  }
  __syncthreads();
  const int64_t e = int64_t(blockIdx.x) * 64 + w * kCW + c;
  const uint64_t boff = uint64_t(e < N ? e : N - 1) * 4u;
  uint32_t key[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    if (j % 16 == 0 && j) __builtin_amdgcn_sched_barrier(0);
    const int q = sub * (R + PAD) + j;
    const uint64_t off = FULL ? boff : (boff & offmask[q]);
    key[j] = __builtin_nontemporal_load(as_global(reinterpret_cast<const uint32_t*>(
        reinterpret_cast<const char*>(rows[q]) + off)));
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < R; ++j) key[j] = f32_key(key[j]);
  // histogram of column c: word (b ^ swz); 4-bin groups stay contiguous and
  // the 16 columns' same bin sit in 16 different banks
  const uint32_t swz = uint32_t(c) * 4u;
  const uint32_t hbase = lds_addr(&hist[c][0]);  // LDS byte address, 1 KB aligned
  const uint32_t bs = hbase | (swz * 4u);
  const uint32_t m3fc = 0x3fcu;
  constexpr uint32_t k_target = KMAX / 2 - 1;
  uint32_t prefix = 0;
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int s = 24 - 8 * pass;
    const uint32_t lo = prefix, hi = prefix | (pass == 0 ? 0xffffffffu : ((2u << (s + 7)) - 1u));
#pragma unroll
    for (int j = 0; j < R; ++j) {
      uint32_t k = key[j];
      if (pass > 0) {
        k = umed3(k, lo, hi);
        key[j] = k;
      }
      const uint32_t sh = s >= 2 ? (k >> (s - 2)) : (k << 2);
      const uint32_t a = and_xor(sh, m3fc, bs);
      lds_add1(a);
    }
    wave_sync();
    // lane (c, sub) owns logical bins [64 sub, 64 sub + 64) = 16 groups of 4
    uint32_t gs[16];
    uint32_t tot = 0;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const u32x4 q = *reinterpret_cast<const u32x4*>(&hist[c][((sub * 16 + g) * 4) ^ swz]);
      gs[g] = q.x + q.y + q.z + q.w;
      tot += gs[g];
    }
    if (pass == 0) {  // ±inf or NaN in the column: bins 0 / 255 hold more than the pads
      const uint32_t b0 = hist[c][0 ^ swz], b255 = hist[c][255 ^ swz];
      if (sub == 0) L.flag[c] = (b0 > uint32_t(below)) || (b255 > uint32_t(KMAX - K - below));
    }
    L.part[c][sub] = tot;
    wave_sync();
    const u32x4 t4 = *reinterpret_cast<const u32x4*>(&L.part[c][0]);
    const uint32_t base = (sub > 0 ? t4.x : 0u) + (sub > 1 ? t4.y : 0u) + (sub > 2 ? t4.z : 0u);
    if (base <= k_target && k_target < base + tot) {
      uint32_t run = base;
      int gsel = 0;
      bool found = false;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const bool hit = !found && run + gs[g] > k_target;
        gsel = hit ? g : gsel;
        run = (!found && !hit) ? run + gs[g] : run;
        found = found || hit;
      }
      const u32x4 q = *reinterpret_cast<const u32x4*>(&hist[c][((sub * 16 + gsel) * 4) ^ swz]);
      int bin = 3;
      if (run + q.x > k_target) bin = 0;
      else if (run + q.x + q.y > k_target) bin = 1;
      else if (run + q.x + q.y + q.z > k_target) bin = 2;
      const uint32_t d = uint32_t((sub * 16 + gsel) * 4 + bin);
      L.pfx[c] = prefix | (d << s);
    }
    wave_sync();
    prefix = L.pfx[c];
    if (pass < 3) {
#pragma unroll
      for (int g = 0; g < 16; ++g)
        *reinterpret_cast<u32x4*>(&hist[c][((sub * 16 + g) * 4) ^ swz]) = u32x4{0, 0, 0, 0};
    }
  }
  uint32_t res = f32_from_key(prefix);
  if (L.flag[c] && sub == 0 && e < N) {  // slow path: the column's first NaN in client order, if any
    for (int q = 0; q < K; ++q) {
      const uint32_t u = reinterpret_cast<const uint32_t*>(src[q])[e];
      if ((u & 0x7fffffffu) > 0x7f800000u) {
        res = u;
        break;
      }
    }
  }
  if (sub == 0 && e < N) reinterpret_cast<uint32_t*>(out)[e] = res;
}

// 16-bit rows, two columns per register (columns 2p, 2p + 1 of pair p in
// the low / high half).  Keys are unsigned 16-bit order keys per half; the
// histogram word of a bin holds the low column's count in bits 0-15 and the
// high column's in bits 16-31 (counts <= 512), so one 256-word histogram
// serves the pair and a ds_add of 1 or 0x10000 counts a half.  Two passes.
struct Bf16Keys {
  static constexpr uint32_t kNegInfKey = 0x007fu, kPosInfKey = 0xff80u;  // keys of 0xff80 / 0x7f80
  static __device__ __forceinline__ bool raw_nan(uint32_t x) { return (x & 0x7fffu) > 0x7f80u; }
};
struct F16Keys {
  static constexpr uint32_t kNegInfKey = 0x03ffu, kPosInfKey = 0xfc00u;  // keys of 0xfc00 / 0x7c00
  static __device__ __forceinline__ bool raw_nan(uint32_t x) { return (x & 0x7fffu) > 0x7c00u; }
};

typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));
typedef short short2_t __attribute__((ext_vector_type(2)));

// order keys of both halves: x ^ 0x8000 (sign clear), ~x (sign set)
__device__ __forceinline__ uint32_t pk_key16(uint32_t r) {
  const uint32_t a = __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2_t, r) >> short(15));
  return r ^ (a | 0x80008000u);
}
__device__ __forceinline__ uint32_t pk_from_key16(uint32_t k) {
  const uint32_t a = __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2_t, k) >> short(15));
  return k ^ (~a | 0x80008000u);
}
__device__ __forceinline__ uint32_t pk_clamp_u16(uint32_t k, uint32_t lo, uint32_t hi) {
  const ushort2_t r = __builtin_elementwise_min(__builtin_elementwise_max(__builtin_bit_cast(ushort2_t, k),
                                                                         __builtin_bit_cast(ushort2_t, lo)),
                                                __builtin_bit_cast(ushort2_t, hi));
  return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ void lds_add(uint32_t a, uint32_t v) {
  __hip_atomic_fetch_add((lds_u32*)(uintptr_t)(a), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// the bin of one half's count that holds rank k (0-based) given the lane's
// 16 group sums gs (packed) and the counts of the lanes below (base)
template <int HALF>
__device__ __forceinline__ uint32_t pk_find_digit(const uint32_t (&gs)[16], uint32_t base, uint32_t k,
                                                  const uint32_t* hrow, uint32_t swz, int sub) {
  uint32_t run = base;
  int gsel = 0;
  bool found = false;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const uint32_t v = HALF ? (gs[g] >> 16) : (gs[g] & 0xffffu);
    const bool hit = !found && run + v > k;
    gsel = hit ? g : gsel;
    run = (!found && !hit) ? run + v : run;
    found = found || hit;
  }
  const u32x4 q = *reinterpret_cast<const u32x4*>(&hrow[((sub * 16 + gsel) * 4) ^ swz]);
  const uint32_t q0 = HALF ? q.x >> 16 : q.x & 0xffffu, q1 = HALF ? q.y >> 16 : q.y & 0xffffu,
                 q2 = HALF ? q.z >> 16 : q.z & 0xffffu;
  int bin = 3;
  if (run + q0 > k) bin = 0;
  else if (run + q0 + q1 > k) bin = 1;
  else if (run + q0 + q1 + q2 > k) bin = 2;
  return uint32_t((sub * 16 + gsel) * 4 + bin);
}

template <int R, bool FULL, class KT>
__global__ __launch_bounds__(256) void median_rsel_pk16_kernel(const uint16_t* const* __restrict__ src, int K,
                                                               int64_t pairs, uint16_t* __restrict__ out,
                                                               const uint32_t* __restrict__ pad2) {
  constexpr int P = 4, KMAX = P * R, PAD = 2;
  __shared__ __attribute__((aligned(1024))) uint32_t hist_all[4][kCW][kBins];
  __shared__ WaveLds lds[4];
  __shared__ uint32_t pfx2[4][kCW][2];
  __shared__ const uint16_t* rows[KMAX + PAD * P];
  __shared__ uint64_t offmask[FULL ? 1 : KMAX + PAD * P];
  const int t = threadIdx.x, w = t >> 6, l = t & 63, c = l & 15, sub = l >> 4;
  if constexpr (FULL) K = KMAX;
  const int below = KMAX / 2 - 1 - (K - 1) / 2;
  for (int i = t; i < KMAX; i += 256) {
    const int q = i + PAD * (i / R);
    if (FULL || i < K) {
      rows[q] = src[i];
      if constexpr (!FULL) offmask[q] = ~uint64_t(0);
    } else {
      rows[q] = reinterpret_cast<const uint16_t*>(&pad2[i - K < below ? 0 : 1]);
      offmask[q] = 0;
    }
  }
  WaveLds& L = lds[w];
  uint32_t (&hist)[kCW][kBins] = hist_all[w];
  {
    uint32_t* h = &hist[0][0];
#pragma unroll
    for (int i = 0; i < 16; ++i) *reinterpret_cast<u32x4*>(h + (i * 64 + l) * 4) = u32x4{0, 0, 0, 0};
  }
  __syncthreads();
  const int64_t e = int64_t(blockIdx.x) * 64 + w * kCW + c;  // column pair
  const uint64_t boff = uint64_t(e < pairs ? e : pairs - 1) * 4u;
  uint32_t key[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    if (j % 16 == 0 && j) __builtin_amdgcn_sched_barrier(0);
    const int q = sub * (R + PAD) + j;
    const uint64_t off = FULL ? boff : (boff & offmask[q]);
    key[j] = __builtin_nontemporal_load(as_global(reinterpret_cast<const uint32_t*>(
        reinterpret_cast<const char*>(rows[q]) + off)));
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < R; ++j) key[j] = pk_key16(key[j]);
  const uint32_t swz = uint32_t(c) * 4u;
  const uint32_t hbase = lds_addr(&hist[c][0]);
  const uint32_t bs = hbase | (swz * 4u);
  const uint32_t m3fc = 0x3fcu;
  constexpr uint32_t k_target = KMAX / 2 - 1;
  uint32_t prefix = 0;  // both halves
  bool special_lo = false, special_hi = false;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1) {
      const uint32_t lo = prefix, hi = prefix | 0x00ff00ffu;
#pragma unroll
      for (int j = 0; j < R; ++j) key[j] = pk_clamp_u16(key[j], lo, hi);
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t k = key[j];
      const uint32_t a_lo = and_xor(pass == 0 ? (k >> 6) : (k << 2), m3fc, bs);
      const uint32_t a_hi = and_xor(pass == 0 ? (k >> 22) : (k >> 14), m3fc, bs);
      lds_add(a_lo, 1u);
      lds_add(a_hi, 0x10000u);
    }
    wave_sync();
    uint32_t gs[16];
    uint32_t tot = 0;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const u32x4 q = *reinterpret_cast<const u32x4*>(&hist[c][((sub * 16 + g) * 4) ^ swz]);
      gs[g] = q.x + q.y + q.z + q.w;
      tot += gs[g];
    }
    if (pass == 0) {  // ±inf / NaN / huge: the outer bins hold more than the pads
      const u32x4 g0 = *reinterpret_cast<const u32x4*>(&hist[c][0 ^ swz]);
      const u32x4 g63 = *reinterpret_cast<const u32x4*>(&hist[c][252 ^ swz]);
      constexpr uint32_t bn = KT::kNegInfKey >> 8, bp = KT::kPosInfKey >> 8;
      uint32_t nlo = g0.x;
      if (bn >= 1) nlo += g0.y;
      if (bn >= 2) nlo += g0.z;
      if (bn >= 3) nlo += g0.w;
      uint32_t nhi = g63.w;
      if (bp <= 254) nhi += g63.z;
      if (bp <= 253) nhi += g63.y;
      if (bp <= 252) nhi += g63.x;
      const uint32_t above = uint32_t(KMAX - K - below);
      special_lo = (nlo & 0xffffu) > uint32_t(below) || (nhi & 0xffffu) > above;
      special_hi = (nlo >> 16) > uint32_t(below) || (nhi >> 16) > above;
    }
    L.part[c][sub] = tot;
    wave_sync();
    const u32x4 t4 = *reinterpret_cast<const u32x4*>(&L.part[c][0]);
    const uint32_t base = (sub > 0 ? t4.x : 0u) + (sub > 1 ? t4.y : 0u) + (sub > 2 ? t4.z : 0u);  // packed
    const uint32_t b_lo = base & 0xffffu, b_hi = base >> 16, t_lo = tot & 0xffffu, t_hi = tot >> 16;
    const int s = 8 - 8 * pass;
    if (b_lo <= k_target && k_target < b_lo + t_lo)
      pfx2[w][c][0] = (prefix & 0xffffu) | (pk_find_digit<0>(gs, b_lo, k_target, hist[c], swz, sub) << s);
    if (b_hi <= k_target && k_target < b_hi + t_hi)
      pfx2[w][c][1] = (prefix >> 16) | (pk_find_digit<1>(gs, b_hi, k_target, hist[c], swz, sub) << s);
    wave_sync();
    prefix = pfx2[w][c][0] | (pfx2[w][c][1] << 16);
    if (pass == 0) {
#pragma unroll
      for (int g = 0; g < 16; ++g)
        *reinterpret_cast<u32x4*>(&hist[c][((sub * 16 + g) * 4) ^ swz]) = u32x4{0, 0, 0, 0};
    }
  }
  uint32_t res = pk_from_key16(prefix);
  if ((special_lo || special_hi) && sub == 0 && e < pairs) {  // first NaN in client order, per half
    bool f_lo = !special_lo, f_hi = !special_hi;
    for (int q = 0; q < K && !(f_lo && f_hi); ++q) {
      const uint32_t u = reinterpret_cast<const uint32_t*>(src[q])[e];
      if (!f_lo && KT::raw_nan(u & 0xffffu)) {
        res = (res & 0xffff0000u) | (u & 0xffffu);
        f_lo = true;
      }
      if (!f_hi && KT::raw_nan(u >> 16)) {
        res = (res & 0xffffu) | (u & 0xffff0000u);
        f_hi = true;
      }
    }
  }
  if (sub == 0 && e < pairs) reinterpret_cast<uint32_t*>(out)[e] = res;
}

// Variant 4: the same selection with PRIVATE per-lane histograms laid out
// bank = lane (word w*64 + lane holds bins 4w..4w+3 of that lane as 8-bit
// counters): the adds of a wave instruction never meet in a bank or an
// address, whatever the data.  The column's count of a bin is the sum of its
// 4 lanes' bytes, taken when the bin's owner lane reads the 4 words.
struct WaveLds2 {
  uint32_t part[kCW][4];
  uint32_t pfx[kCW];
  uint32_t flag[kCW][4];
};

template <int R, bool FULL>
__global__ __launch_bounds__(256) void median_rsel2_f32_kernel(const float* const* __restrict__ src, int K, int64_t N,
                                                               float* __restrict__ out) {
  constexpr int P = 4, KMAX = P * R, PAD = 2;
  __shared__ __attribute__((aligned(16384))) uint32_t hist_all[4][64 * 64];  // [wave][word w * 64 + lane]
  __shared__ WaveLds2 lds[4];
  __shared__ const float* rows[KMAX + PAD * P];
  __shared__ uint64_t offmask[FULL ? 1 : KMAX + PAD * P];
  const int t = threadIdx.x, w = t >> 6, l = t & 63, c = l & 15, sub = l >> 4;
  if constexpr (FULL) K = KMAX;
  const int below = KMAX / 2 - 1 - (K - 1) / 2;
  for (int i = t; i < KMAX; i += 256) {
    const int q = i + PAD * (i / R);
    if (FULL || i < K) {
      rows[q] = src[i];
      if constexpr (!FULL) offmask[q] = ~uint64_t(0);
    } else {
      rows[q] = &g_pad_f32[i - K < below ? 0 : 1];
      offmask[q] = 0;
    }
  }
  WaveLds2& L = lds[w];
  uint32_t* hist = hist_all[w];
#pragma unroll
  for (int i = 0; i < 16; ++i) *reinterpret_cast<u32x4*>(hist + (i * 64 + l) * 4) = u32x4{0, 0, 0, 0};
  __syncthreads();
  const int64_t e = int64_t(blockIdx.x) * 64 + w * kCW + c;
  const uint64_t boff = uint64_t(e < N ? e : N - 1) * 4u;
  uint32_t key[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    if (j % 16 == 0 && j) __builtin_amdgcn_sched_barrier(0);
    const int q = sub * (R + PAD) + j;
    const uint64_t off = FULL ? boff : (boff & offmask[q]);
    key[j] = __builtin_nontemporal_load(as_global(reinterpret_cast<const uint32_t*>(
        reinterpret_cast<const char*>(rows[q]) + off)));
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < R; ++j) key[j] = f32_key(key[j]);
  const uint32_t lb = lds_addr(hist) + uint32_t(l) * 4u;  // 16 KB-aligned wave base | lane
  const uint32_t m3f00 = 0x3f00u;
  constexpr uint32_t k_target = KMAX / 2 - 1;
  const uint32_t above = uint32_t(KMAX - K - below);
  uint32_t prefix = 0;
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int s = 24 - 8 * pass;
    const uint32_t lo = prefix, hi = prefix | (pass == 0 ? 0xffffffffu : ((2u << (s + 7)) - 1u));
#pragma unroll
    for (int j = 0; j < R; ++j) {
      uint32_t k = key[j];
      if (pass > 0) {
        k = umed3(k, lo, hi);
        key[j] = k;
      }
      const uint32_t a = and_or(s >= 6 ? (k >> (s - 6)) : (k << 6), m3f00, lb);
      const uint32_t inc = 1u << ((s >= 3 ? (k >> (s - 3)) : (k << 3)) & 0x18u);
      lds_add(a, inc);
    }
    wave_sync();
    // lane (c, sub): words 16 sub .. 16 sub + 15 of the column's 4 lanes
    // (lanes s' * 16 + c); E = bins 4w, 4w+2 and O = bins 4w+1, 4w+3 as
    // 16-bit fields summed over the 4 lanes; the words are zeroed behind
    uint32_t E[16], O[16];
    uint32_t tot = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint32_t* wp = hist + (16 * sub + j) * 64 + c;
      const uint32_t x0 = wp[0], x1 = wp[16], x2 = wp[32], x3 = wp[48];
      wp[0] = 0u;
      wp[16] = 0u;
      wp[32] = 0u;
      wp[48] = 0u;
      E[j] = (x0 & 0x00ff00ffu) + (x1 & 0x00ff00ffu) + (x2 & 0x00ff00ffu) + (x3 & 0x00ff00ffu);
      O[j] = ((x0 >> 8) & 0x00ff00ffu) + ((x1 >> 8) & 0x00ff00ffu) + ((x2 >> 8) & 0x00ff00ffu) +
             ((x3 >> 8) & 0x00ff00ffu);
      const uint32_t g = E[j] + O[j];
      tot += (g & 0xffffu) + (g >> 16);
    }
    if (pass == 0) {  // ±inf / NaN / huge: bins 0 and 255 hold more than the pads
      const bool sp = (sub == 0 && (E[0] & 0xffffu) > uint32_t(below)) || (sub == 3 && (O[15] >> 16) > above);
      L.flag[c][sub] = sp;
    }
    L.part[c][sub] = tot;
    wave_sync();
    const u32x4 t4 = *reinterpret_cast<const u32x4*>(&L.part[c][0]);
    const uint32_t base = (sub > 0 ? t4.x : 0u) + (sub > 1 ? t4.y : 0u) + (sub > 2 ? t4.z : 0u);
    if (base <= k_target && k_target < base + tot) {
      uint32_t run = base, ew = 0, ow = 0;
      int jsel = 0;
      bool found = false;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint32_t g = E[j] + O[j];
        const uint32_t v = (g & 0xffffu) + (g >> 16);
        const bool hit = !found && run + v > k_target;
        jsel = hit ? j : jsel;
        ew = hit ? E[j] : ew;
        ow = hit ? O[j] : ow;
        run = (!found && !hit) ? run + v : run;
        found = found || hit;
      }
      const uint32_t b0 = ew & 0xffffu, b1 = ow & 0xffffu, b2 = ew >> 16;
      int bin = 3;
      if (run + b0 > k_target) bin = 0;
      else if (run + b0 + b1 > k_target) bin = 1;
      else if (run + b0 + b1 + b2 > k_target) bin = 2;
      L.pfx[c] = prefix | (uint32_t((16 * sub + jsel) * 4 + bin) << s);
    }
    wave_sync();
    prefix = L.pfx[c];
  }
  uint32_t res = f32_from_key(prefix);
  const u32x4 f4 = *reinterpret_cast<const u32x4*>(&L.flag[c][0]);
  if ((f4.x | f4.w) && sub == 0 && e < N) {  // slow path: the column's first NaN in client order, if any
    for (int q = 0; q < K; ++q) {
      const uint32_t u = reinterpret_cast<const uint32_t*>(src[q])[e];
      if ((u & 0x7fffffffu) > 0x7f800000u) {
        res = u;
        break;
      }
    }
  }
  if (sub == 0 && e < N) reinterpret_cast<uint32_t*>(out)[e] = res;
}

__device__ uint32_t g_pad_bf16x2[2] = {0xff80ff80u, 0x7f807f80u};
__device__ uint32_t g_pad_f16x2[2] = {0xfc00fc00u, 0x7c007c00u};

extern "C" int rsel_launch(int variant, const void* src, int K, int64_t N, void* out, void* stream) {
  const int64_t grid = (N + 63) / 64;
  auto st = reinterpret_cast<hipStream_t>(stream);
  auto s = reinterpret_cast<const float* const*>(src);
  auto o = reinterpret_cast<float*>(out);
  if (variant == 0) {
    if (K <= 256 || K > 512) return -1;
    if (K == 512)
      hipLaunchKernelGGL((median_rsel_f32_kernel<128, true>), dim3(unsigned(grid)), dim3(256), 0, st, s, K, N, o);
    else
      hipLaunchKernelGGL((median_rsel_f32_kernel<128, false>), dim3(unsigned(grid)), dim3(256), 0, st, s, K, N, o);
  } else if (variant == 1) {
    if (K <= 128 || K > 256) return -1;
    if (K == 256)
      hipLaunchKernelGGL((median_rsel_f32_kernel<64, true>), dim3(unsigned(grid)), dim3(256), 0, st, s, K, N, o);
    else
      hipLaunchKernelGGL((median_rsel_f32_kernel<64, false>), dim3(unsigned(grid)), dim3(256), 0, st, s, K, N, o);
  } else if (variant == 4) {
    if (K <= 256 || K > 512) return -1;
    if (K == 512)
      hipLaunchKernelGGL((median_rsel2_f32_kernel<128, true>), dim3(unsigned(grid)), dim3(256), 0, st, s, K, N, o);
    else
      hipLaunchKernelGGL((median_rsel2_f32_kernel<128, false>), dim3(unsigned(grid)), dim3(256), 0, st, s, K, N, o);
  } else if (variant == 2 || variant == 3) {  // bf16 / f16 rows, even N, K in (256, 512]
    if (K <= 256 || K > 512 || (N & 1)) return -1;
    const int64_t pairs = N / 2, g2 = (pairs + 63) / 64;
    auto s16 = reinterpret_cast<const uint16_t* const*>(src);
    auto o16 = reinterpret_cast<uint16_t*>(out);
    uint32_t* pad = nullptr;
    if (hipGetSymbolAddress(reinterpret_cast<void**>(&pad), variant == 2 ? HIP_SYMBOL(g_pad_bf16x2)
                                                                         : HIP_SYMBOL(g_pad_f16x2)) != hipSuccess)
      return -4;
    if (variant == 2) {
      if (K == 512)
        hipLaunchKernelGGL((median_rsel_pk16_kernel<128, true, Bf16Keys>), dim3(unsigned(g2)), dim3(256), 0, st, s16,
                           K, pairs, o16, pad);
      else
        hipLaunchKernelGGL((median_rsel_pk16_kernel<128, false, Bf16Keys>), dim3(unsigned(g2)), dim3(256), 0, st,
                           s16, K, pairs, o16, pad);
    } else {
      if (K == 512)
        hipLaunchKernelGGL((median_rsel_pk16_kernel<128, true, F16Keys>), dim3(unsigned(g2)), dim3(256), 0, st, s16,
                           K, pairs, o16, pad);
      else
        hipLaunchKernelGGL((median_rsel_pk16_kernel<128, false, F16Keys>), dim3(unsigned(g2)), dim3(256), 0, st,
                           s16, K, pairs, o16, pad);
    }
  } else {
    return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
