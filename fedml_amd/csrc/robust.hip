// robust.hip — gfx950 kernels for FedML's distance-based robust aggregation
// (the Krum / multi-Krum and norm-difference-clipping defenses), exported
// through include/fedagg.h and linked into libfedagg.so beside fedagg.hip.
//
// What this replaces (python/fedml/core/security/):
//   defense/krum_defense.py:47-60          K(K-1) torch norms of client differences
//   defense/norm_diff_clipping_defense.py:20-54   one norm per client + the clipped rebuild
//   defense/cclip_defense.py:30-80         bucket distances to the guess + the scaled differences
//   common/utils.py:8-13, 24-27            vectorize_weight / compute_euclidean_distance
//
// Rows are K device pointers (client updates laid out as bucket rows); the
// columns that count ("weight" keys, common/utils.py:16-21) arrive as a chunk
// table of (start, length) pairs built on the host from the key segments.
//
//   fedagg_dist2_f32     out[i] = sum_e (x_i[e] - r[e])^2        (HBM-bound, one pass)
//   fedagg_pairdist2_f32 out[i][j] = sum_e (x_i[e] - x_j[e])^2   (VALU-bound, packed fp32)
//   fedagg_clip_diff_f32 y_i[e] = fl(fl(fl(x_i[e] - r[e]) / c_i) + r[e])
//   fedagg_scale_diff_f32 y_i[e] = fl(fl(x_i[e] - r[e]) * s_i)   (CClip)
//
// Every difference is the fp32 difference the reference forms
// (vec_local - vec_global, v1 - v2).  dist2 squares it exactly in fp64 and sums
// in fp64: the exact sum up to fp64 rounding.  pairdist2 squares and sums in
// packed fp32 over a stage of at most 64 columns (relative error ~sqrt(64)
// ulp typical, 64 ulp at worst) and adds the stage sums in fp64: about the
// accuracy of the reference's own fp32 torch.norm (~1e-7 relative).
// Partial sums go to a workspace and are combined in a fixed order: results
// are deterministic run to run.

#include <hip/hip_runtime.h>

#include <type_traits>
#include <stdint.h>

#include <string>

#include "../../include/fedagg.h"


extern "C" int fedagg_set_error_internal(int code, const char* msg);

namespace {

int rset(int code, const std::string& msg) { return fedagg_set_error_internal(code, msg.c_str()); }

int rcheck(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return rset(static_cast<int>(e), std::string(what) + ": " + hipGetErrorString(e));
  return FEDAGG_OK;
}

template <class T>
__device__ __forceinline__ const T __attribute__((address_space(1)))* gptr(const T* p) {
  return (const T __attribute__((address_space(1)))*)(p);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kBS = 256;
constexpr int kWaves = kBS / 64;
constexpr int kLaneCols = FEDAGG_DIST_CHUNK / 64;  // columns per lane per chunk (kLaneCols / 4 f32x4)
// clients per wave per pass of dist2_kernel (kWaves * kBatch per block).  32
// would cover 128 clients in one pass but costs the occupancy: 2.61 vs 1.99 ms
// at config 3 (tools/robust_variants.py, profiles/r03/dist/); with the
// reference row cached in L2 (ld4<false>) the second pass's re-read is cheap
constexpr int kBatch = 16;  // dist2: clients per batch (16 vs 32: profiles/r03/dist/)

// A workgroup barrier that waits for this wave's LDS operations only.
// __syncthreads() carries a release fence that waits for EVERY outstanding
// memory operation (s_waitcnt vmcnt(0) lgkmcnt(0) before s_barrier), so the
// next stage's global loads, issued just before it, were drained at every
// barrier instead of overlapping the stage's compute.  The "memory" clobber
// keeps the compiler from moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// Columns lane*4 + 256*u (u < kLaneCols/4) of a chunk of `len` columns at
// `p`: 16-byte loads where a whole f32x4 lies in the chunk and p is 16-byte
// aligned (bucket rows and key offsets are), 4-byte loads otherwise; columns
// past len read 0.
// NT = false for a row every wave of the block reads (the reference row):
// a plain load leaves it in L2 for the other three waves; non-temporal loads
// made each wave fetch it from HBM again (dist2's traffic was 1.05x the
// algorithmic bytes, ~7 extra reference rows per call at config 3)
template <bool NT = true>
__device__ __forceinline__ f32x4 ld4(const float* p) {
  const auto q = reinterpret_cast<const f32x4 __attribute__((address_space(1)))*>(gptr(p));
  if constexpr (NT) return __builtin_nontemporal_load(q);
  return *q;
}

template <bool NT = true>
__device__ __forceinline__ void load_chunk(const float* p, int len, int lane, f32x4 (&v)[kLaneCols / 4]) {
  const bool al = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  if (al && len == FEDAGG_DIST_CHUNK) {  // wave-uniform: a full aligned chunk, no per-lane conditions
#pragma unroll
    for (int u = 0; u < kLaneCols / 4; ++u) v[u] = ld4<NT>(p + lane * 4 + 256 * u);
    return;
  }
#pragma unroll
  for (int u = 0; u < kLaneCols / 4; ++u) {
    const int c = lane * 4 + 256 * u;
    if (al && c + 4 <= len) {
      v[u] = ld4<NT>(p + c);
    } else {
      v[u].x = c < len ? gptr(p)[c] : 0.f;
      v[u].y = c + 1 < len ? gptr(p)[c + 1] : 0.f;
      v[u].z = c + 2 < len ? gptr(p)[c + 2] : 0.f;
      v[u].w = c + 3 < len ? gptr(p)[c + 3] : 0.f;
    }
  }
}

__device__ __forceinline__ double sq_diff(float x, float r, double acc) {
  const float d = x - r;  // the reference's fp32 difference
  return __builtin_fma(double(d), double(d), acc);  // exact square, fp64 sum
}

// ---------------------------------------------------------------------------
// Per-client squared distance to a reference row.  A block owns the chunks
// g, g + G, ... (a column range) for every client: per chunk each lane holds
// its reference columns in registers, and wave w streams clients
// w, w + 4, ... (kBatch of them per pass, one fp64 accumulator each) against
// them.  The reference row is read from HBM once per pass, not once per
// client (a client-major grid re-read it ~57x: 1.43x the algorithmic bytes).
__global__ __launch_bounds__(kBS) void dist2_kernel(const float* const* __restrict__ src, int K,
                                                    const float* __restrict__ ref, const int64_t* __restrict__ chunks,
                                                    int64_t n_chunks, int G, double* __restrict__ partial) {
  const int g = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int cb = 0; cb < K; cb += kWaves * kBatch) {
    double acc[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) acc[j] = 0.0;
    for (int64_t c = g; c < n_chunks; c += G) {
      const int64_t start = chunks[2 * c];
      const int len = int(chunks[2 * c + 1]);
      f32x4 r[kLaneCols / 4];
      if (ref) {
        load_chunk<false>(ref + start, len, lane, r);
      } else {
#pragma unroll
        for (int u = 0; u < kLaneCols / 4; ++u) r[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const int i = cb + w + kWaves * j;
        if (i < K) {  // wave-uniform
          f32x4 x[kLaneCols / 4];
          load_chunk<true>(src[i] + start, len, lane, x);
#pragma unroll
          for (int u = 0; u < kLaneCols / 4; ++u) {
            acc[j] = sq_diff(x[u].x, r[u].x, acc[j]);
            acc[j] = sq_diff(x[u].y, r[u].y, acc[j]);
            acc[j] = sq_diff(x[u].z, r[u].z, acc[j]);
            acc[j] = sq_diff(x[u].w, r[u].w, acc[j]);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const int i = cb + w + kWaves * j;
      if (i < K) {
        const double t = wave_sum(acc[j]);
        if (lane == 0) partial[int64_t(i) * G + g] = t;
      }
    }
  }
}

// out[i] = sum over g of partial[i][g]: one block per row, thread t sums
// g = t, t + 256, ... in order, then a fixed LDS tree (deterministic).  The
// first version, one thread per row summing all G in sequence, was a chain of
// G dependent loads: 0.218 ms per call at config 3 (G = 1,024), a tenth of
// the whole dist2 call.
__global__ __launch_bounds__(256) void sum_rows_kernel(const double* __restrict__ partial, int G,
                                                       double* __restrict__ out) {
  __shared__ double red[256];
  const int i = blockIdx.x, t = threadIdx.x;
  const double* p = partial + int64_t(i) * G;
  double s = 0.0;
  for (int g = t; g < G; g += 256) s += p[g];
  red[t] = s;
  __syncthreads();
#pragma unroll
  for (int m = 128; m > 0; m >>= 1) {
    if (t < m) red[t] += red[t + m];
    __syncthreads();
  }
  if (t == 0) out[i] = red[0];
}

// ---------------------------------------------------------------------------
// Pairwise squared distances.  The K x K pair matrix is cut into 64 x 64
// client tiles (I <= J); a block owns one tile over the chunk group g.  Per
// stage of 64 columns each wave loads 16 client rows of tile I (and of J) as
// coalesced 256-B row segments into registers one stage ahead, then writes
// them four rows at a time as one 16-byte LDS write per lane: sX[column][client], rows padded by one group so
// both the staging writes and the compute reads are bank-conflict free.  Thread (ti, tj) then owns clients 4ti..4ti+3 of I x 4tj..4tj+3 of J:
// per column one 16-byte LDS read per side and 16 squared differences, as 8
// packed fp32 subtracts and 8 packed fp32 FMAs (v_pk_add_f32 / v_pk_fma_f32).
// fp32 sums over one stage (<= 64 columns) are flushed into fp64
// accumulators, which go to the workspace per block.
constexpr int kPT = 64;      // clients per tile side
constexpr int kStage = 64;   // columns per LDS stage

// [column][client] tile rows padded by one 4-client group (272 B): a staging
// write (lane = column, 16 B) walks the banks 16 B apart, and a compute read's
// address is the thread's group base plus a constant per unrolled column (an
// immediate offset; the earlier XOR swizzle cost two VALU ops per column)
constexpr int kRowF = kPT + 4;
__device__ __forceinline__ int swz(int c, int grp) { return c * kRowF + (grp << 2); }

// The 16 client rows (4 groups of 4) a wave stages for one 64-client side:
// wave-uniform pointers, read once per block (kept in SGPRs); a row past K
// points at row 0 and is zeroed by `live`.
struct SideRows {
  const float* p[4][4];
  bool live[4][4];
};

__device__ __forceinline__ SideRows side_rows(const float* const* __restrict__ src, int K, int base, int wave) {
  SideRows r;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int cl = base + (wave * 4 + q) * 4 + k;
      r.live[q][k] = cl < K;
      r.p[q][k] = src[cl < K ? cl : 0];
    }
  return r;
}

// A stage's global loads for one side, into registers (lane = column):
// unconditional loads at a clamped column, then zeroed past w / past K, so
// all 16 are in flight together.  Issued one stage ahead, they overlap the
// current stage's compute.
__device__ __forceinline__ void stage_load(f32x4 (&v)[4], const SideRows& rows, int64_t col0, int w, int lane) {
  const int c = lane < w ? lane : 0;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int k = 0; k < 4; ++k) v[q][k] = __builtin_nontemporal_load(gptr(rows.p[q][k]) + col0 + c);
}

// the staged values, zeroed past column w and past K: a mask applied here,
// when the stage is written to LDS, not right after the loads, so nothing
// consumes them early and they stay in flight through the current stage's
// compute (a select on the uniform `live` had become a branch around each
// load with a full vmcnt(0) wait at every join)
__device__ __forceinline__ void stage_store(f32x4* __restrict__ s, const f32x4 (&v)[4], const SideRows& rows, int w,
                                            int t) {
  const int lane = t & 63, wave = t >> 6;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x4 x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t m = (rows.live[q][k] && lane < w) ? 0xffffffffu : 0u;
      x[k] = __uint_as_float(__float_as_uint(v[q][k]) & m);
    }
    s[swz(lane, wave * 4 + q) >> 2] = x;
  }
}

// one column of the thread's 4 x 4 pair block: acc[2k + h] holds pairs
// (4ti + k, 4tj + 2h) and (4ti + k, 4tj + 2h + 1); a = the column's values of
// clients 4ti.., b = of clients 4tj..
__device__ __forceinline__ void pair_ab(f32x4 a, f32x4 b, f32x2 (&acc)[8]) {
  const f32x2 b01 = {b[0], b[1]}, b23 = {b[2], b[3]};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x2 ak = {a[k], a[k]};
    const f32x2 d0 = ak - b01, d1 = ak - b23;  // v_pk_add_f32 (neg, op_sel broadcast)
    acc[2 * k] = __builtin_elementwise_fma(d0, d0, acc[2 * k]);  // v_pk_fma_f32
    acc[2 * k + 1] = __builtin_elementwise_fma(d1, d1, acc[2 * k + 1]);
  }
}

// The columns [0, w) of a stage; pa / pb point at column 0 of the thread's
// two 4-client groups, RS = row stride in f32x4.  A full stage reads column
// c + 1 before column c computes (the last prefetch reads a pad row past the
// stage), so a wave does not wait a whole LDS round trip in front of every
// column: SQ_WAIT_ANY was 52 % of the triangle kernel's wave cycles.
template <int RS>
__device__ __forceinline__ void pair_stage(const f32x4* pa, const f32x4* pb, int w, f32x2 (&acc)[8]) {
  if (w == kStage) {
    f32x4 an = pa[0], bn = pb[0];
#pragma unroll 8
    for (int col = 0; col < kStage; ++col) {
      const f32x4 a = an, b = bn;
      an = pa[(col + 1) * RS];
      bn = pb[(col + 1) * RS];
      __builtin_amdgcn_sched_barrier(0);  // keep the scheduler from sinking the prefetch to its use
      pair_ab(a, b, acc);
    }
  } else {
    for (int col = 0; col < w; ++col) pair_ab(pa[col * RS], pb[col * RS], acc);
  }
}

// tile pair tp -> (a, b), a <= b, row-major over the upper triangle of T x T
__device__ __forceinline__ int2 tile_of(int tp, int T) {
  int a = 0;
  while (tp >= T - a) {
    tp -= T - a;
    ++a;
  }
  return int2{a, a + tp};
}

__global__ __launch_bounds__(kBS) void pairdist_kernel(const float* const* __restrict__ src, int K,
                                                       const int64_t* __restrict__ chunks, int64_t n_chunks, int G,
                                                       double* __restrict__ partial) {
  __shared__ f32x4 sA[(kStage + 1) * kRowF / 4];  // + the pad row pair_stage's last prefetch reads
  __shared__ f32x4 sB[(kStage + 1) * kRowF / 4];
  const int tp = blockIdx.x, g = blockIdx.y, t = threadIdx.x;
  const int2 tile = tile_of(tp, (K + kPT - 1) / kPT);
  const int I = tile.x * kPT, J = tile.y * kPT;
  const bool diag = tile.x == tile.y;
  const f32x4* sJ = diag ? sA : sB;
  const int ti = t >> 4, tj = t & 15;
  double acc64[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) acc64[k] = 0.0;
  // the stages of chunks g, g + G, ... in order; (c, s0) is the next stage
  int64_t c = g;
  int s0 = 0;
  const int lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const SideRows rowsA = side_rows(src, K, I, wave);
  const SideRows rowsB = side_rows(src, K, diag ? I : J, wave);
  f32x4 va[4], vb[4];
  int64_t col_next = 0;
  int w_next = 0;
  auto fetch = [&]() {  // issue the next stage's loads; false past the last stage
    if (c >= n_chunks) return false;
    const int len = int(chunks[2 * c + 1]);
    col_next = chunks[2 * c] + s0;
    w_next = len - s0 < kStage ? len - s0 : kStage;
    stage_load(va, rowsA, col_next, w_next, lane);
    if (!diag) stage_load(vb, rowsB, col_next, w_next, lane);
    s0 += kStage;
    if (s0 >= len) {
      s0 = 0;
      c += G;
    }
    return true;
  };
  bool have = fetch();
  while (have) {
    const int w = w_next;
    lds_barrier();  // the previous stage's LDS reads are done
    stage_store(sA, va, rowsA, w, t);
    if (!diag) stage_store(sB, vb, rowsB, w, t);
    have = fetch();  // next stage's loads in flight during this stage's compute
    lds_barrier();
    f32x2 acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = f32x2{0.f, 0.f};
    pair_stage<kRowF / 4>(sA + (swz(0, ti) >> 2), sJ + (swz(0, tj) >> 2), w, acc);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      acc64[2 * k] += double(acc[k][0]);
      acc64[2 * k + 1] += double(acc[k][1]);
    }
  }
  // pair (4ti + k, 4tj + m) of the tile at acc64[4k + m]
  double* out = partial + (int64_t(tp) * G + g) * (kPT * kPT);
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int m = 0; m < 4; ++m) out[(4 * ti + k) * kPT + 4 * tj + m] = acc64[4 * k + m];
}

// D[a][b] and D[b][a] from the tiles' partials.  A block owns 64 pairs of a
// tile (one coalesced 512-B row of the partials per chunk group); its four
// waves sum the chunk groups g = q, q + 4, ... (8 loads in flight per lane),
// and the four quarter sums are added in a fixed order: deterministic.  (One
// thread per pair summing all G in sequence kept 16 blocks per tile busy:
// 0.33 ms at config 3.)
__global__ __launch_bounds__(256) void pair_finish_kernel(const double* __restrict__ partial, int G, int K,
                                                          double* __restrict__ D) {
  __shared__ double quarter[4][64];
  const int tp = blockIdx.y, lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;  // pair index in the tile
  const double* p = partial + int64_t(tp) * G * (kPT * kPT) + e;
  double s[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int g = q;
  for (; g + 28 < G; g += 32) {
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += p[int64_t(g + 4 * u) * (kPT * kPT)];
  }
#pragma unroll
  for (int u = 0; u < 8; ++u)  // the last < 8 of this quarter's groups
    if (g + 4 * u < G) s[u] += p[int64_t(g + 4 * u) * (kPT * kPT)];
  quarter[q][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (q != 0) return;
  const double t = (quarter[0][lane] + quarter[1][lane]) + (quarter[2][lane] + quarter[3][lane]);
  const int2 tile = tile_of(tp, (K + kPT - 1) / kPT);
  const int a = tile.x * kPT + e / kPT, b = tile.y * kPT + e % kPT;
  if (a >= K || b >= K) return;
  D[int64_t(a) * K + b] = a == b ? 0.0 : t;
  if (tile.x != tile.y) D[int64_t(b) * K + a] = t;
}

// ---------------------------------------------------------------------------
// Up to 128 clients: the pair triangle in ONE block per chunk group.  The
// tiled kernel above runs a 64 x 64 diagonal tile as a full square (256 4x4
// pair blocks for the 136 of its upper triangle): at K = 128 that is 768
// block-threads for 528 useful blocks, at K = 64 256 for 136.  Here every
// client sits in LDS per stage (128 clients x 64 columns = 33 KB,
// [column][client], rows padded by one 4-client group) and thread t owns
// the t-th 4x4 block (bi <= bj, row-major) of the upper triangle: 576 threads
// (9 waves) at K = 128, 192 at K = 64.  Per column and thread the work is the
// tiled kernel's (two 16-byte LDS reads, 8 packed subtracts, 8 packed FMAs,
// fp32 stage sums flushed into fp64).  A diagonal block computes all 16
// slots; its mirrored halves are the same fp32 values.  Partials are laid out
// [g][slot][block] so both their stores and the finish kernel's reads are
// coalesced.
constexpr int kTriMax = 128;   // clients the triangle kernel holds
constexpr int kTriBS = 576;    // 9 waves: 528 blocks at K = 128
constexpr int kTriLoads = 6;   // 4-client groups a wave stages per stage

// rows of NB 4-client groups padded by one group (an odd number of 16-byte
// slots: conflict-free staging writes, as the tiles' rows); the kernel is
// instantiated for NB = 16 (K <= 64) and 32 (K <= 128) so its two stage
// buffers take 35 / 69 KB of LDS
template <int NB>
constexpr int tri_row_f() { return 4 * (NB + 1); }
template <int NB>
__device__ __forceinline__ int tri_swz(int c, int grp) { return c * tri_row_f<NB>() + (grp << 2); }

__host__ __device__ inline int tri_blocks(int K) {
  const int nb = (K + 3) / 4;
  return nb * (nb + 1) / 2;
}
// threads of the triangle kernel: every block owned, every 4-client group staged
inline int tri_threads(int K) {
  const int nb = (K + 3) / 4, nblk = tri_blocks(K);
  int w = (nblk + 63) / 64;
  const int wl = (nb + kTriLoads - 1) / kTriLoads;
  return 64 * (w > wl ? w : wl);
}

// block index -> (bi, bj), row-major over the upper triangle of nb x nb
__device__ __forceinline__ int2 tri_block(int t, int nb) {
  int bi = 0;
  while (t >= nb - bi) {
    t -= nb - bi;
    ++bi;
  }
  return int2{bi, bi + t};
}

template <int NBMAX>
__global__ __launch_bounds__(kTriBS) void pairtri_kernel(const float* const* __restrict__ src, int K,
                                                        const int64_t* __restrict__ chunks, int64_t n_chunks, int G,
                                                        double* __restrict__ partial) {
  // two stage buffers (one barrier per stage), each with the pad row
  // pair_stage's last prefetch reads
  __shared__ f32x4 sX[2][(kStage + 1) * tri_row_f<NBMAX>() / 4];
  const int g = blockIdx.x, t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6), W = blockDim.x >> 6;
  const int nb = (K + 3) >> 2, nblk = nb * (nb + 1) / 2;
  const bool active = t < nblk;
  const int2 blk = tri_block(active ? t : 0, nb);
  // the groups this wave stages: wave, wave + W, ... (wave-uniform pointers
  // in SGPRs; a row past K points at row 0 and is zeroed by the mask)
  const float* rp[kTriLoads][4];
  bool live[kTriLoads][4];
#pragma unroll
  for (int q = 0; q < kTriLoads; ++q)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int cl = 4 * (wave + W * q) + k;
      live[q][k] = cl < K;
      rp[q][k] = src[cl < K ? cl : 0];
    }
  double acc64[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) acc64[k] = 0.0;
  int64_t c = g;
  int s0 = 0;
  f32x4 v[kTriLoads];
  int w_next = 0;
  auto fetch = [&]() {  // the next stage's loads; false past the last stage
    if (c >= n_chunks) return false;
    const int len = int(chunks[2 * c + 1]);
    const int64_t col0 = chunks[2 * c] + s0;
    w_next = len - s0 < kStage ? len - s0 : kStage;
    const int cc = lane < w_next ? lane : 0;
#pragma unroll
    for (int q = 0; q < kTriLoads; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[q][k] = __builtin_nontemporal_load(gptr(rp[q][k]) + col0 + cc);
    s0 += kStage;
    if (s0 >= len) {
      s0 = 0;
      c += G;
    }
    return true;
  };
  // the staged registers -> a stage buffer, zeroed past the stage's width w
  // and past K here (not in fetch: the loads stay in flight until now)
  auto stage_to = [&](f32x4* buf, int w) {
#pragma unroll
    for (int q = 0; q < kTriLoads; ++q)
      if (wave + W * q < nb) {
        f32x4 x;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t m = (live[q][k] && lane < w) ? 0xffffffffu : 0u;
          x[k] = __uint_as_float(__float_as_uint(v[q][k]) & m);
        }
        buf[tri_swz<NBMAX>(lane, wave + W * q) >> 2] = x;
      }
  };
  // Stage s computes from buffer s & 1 while stage s + 1 is written into the
  // other one and stage s + 2's loads are in flight: one barrier per stage.
  // A buffer is rewritten only after the barrier that ends its readers' stage.
  bool have = fetch();
  if (have) {
    int w = w_next;
    stage_to(sX[0], w);
    have = fetch();
    lds_barrier();
    for (int buf = 0;; buf ^= 1) {
      if (active) {
        f32x2 acc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = f32x2{0.f, 0.f};
        pair_stage<tri_row_f<NBMAX>() / 4>(sX[buf] + (tri_swz<NBMAX>(0, blk.x) >> 2),
                                           sX[buf] + (tri_swz<NBMAX>(0, blk.y) >> 2), w, acc);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          acc64[2 * k] += double(acc[k][0]);
          acc64[2 * k + 1] += double(acc[k][1]);
        }
      }
      if (!have) break;
      const int wn = w_next;
      stage_to(sX[buf ^ 1], wn);
      have = fetch();
      lds_barrier();
      w = wn;
    }
  }
  if (active) {
    double* out = partial + int64_t(g) * 16 * nblk + t;
#pragma unroll
    for (int j = 0; j < 16; ++j) out[int64_t(j) * nblk] = acc64[j];  // slot j = 4k + m: pair (4bi + k, 4bj + m)
  }
}

// D from the triangle kernel's partials: entry e = slot * nblk + block, the
// chunk groups summed in four fixed-order quarters as in pair_finish_kernel
__global__ __launch_bounds__(256) void tri_finish_kernel(const double* __restrict__ partial, int G, int K,
                                                         double* __restrict__ D) {
  __shared__ double quarter[4][64];
  const int nb = (K + 3) >> 2, nblk = nb * (nb + 1) / 2, E = 16 * nblk;
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  const int ec = e < E ? e : E - 1;
  const double* p = partial + ec;
  double s[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int g = q;
  for (; g + 28 < G; g += 32) {
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += p[int64_t(g + 4 * u) * E];
  }
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (g + 4 * u < G) s[u] += p[int64_t(g + 4 * u) * E];
  quarter[q][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (q != 0 || e >= E) return;
  const double tsum = (quarter[0][lane] + quarter[1][lane]) + (quarter[2][lane] + quarter[3][lane]);
  const int j = e / nblk;
  const int2 blk = tri_block(e - j * nblk, nb);
  const int a = 4 * blk.x + (j >> 2), b = 4 * blk.y + (j & 3);
  if (a >= K || b >= K) return;
  // a diagonal block holds (a, b) and (b, a) as equal values: both write both
  D[int64_t(a) * K + b] = a == b ? 0.0 : tsum;
  D[int64_t(b) * K + a] = a == b ? 0.0 : tsum;
}

// ---------------------------------------------------------------------------
// Pairwise squared distances as a CENTRED Gram on fp32 MFMA (K <= 128).
//
// D_ij = sum_e (x_i[e] - x_j[e])^2 = sum_e (c_i[e] - c_j[e])^2 with c = x - r
// for ANY per-column r, so D = G_ii + G_jj - 2 G_ij over the Gram G of the
// centred rows: one FMA per client pair and column on the matrix cores
// (v_mfma_f32_16x16x4_f32) instead of the exact-difference kernel's packed
// subtract + packed FMA on the VALU.  Centring is what keeps the Gram form
// accurate: honest clients are close to one another (base + small
// updates), so uncentred |x|^2 would dwarf D and cancel.  Per 64-column stage
// r is the column mean over the K clients, so |c|^2 is of the order of the
// distances themselves.
//
// Layout: a block owns chunk groups g, g + G, ... (like pairtri_kernel); per
// stage its 4 waves stage all NB*16 client rows of 64 columns into LDS
// ([client][column], rows of kGramRS floats; lane = column, so every global
// load is one coalesced 256-B row segment with a wave-uniform base) and
// write per-wave column sums beside them.  After one barrier each wave
// builds, for each of its tiles (a 16 x 16 block of the client-group
// triangle, row-major, a wave owning a contiguous run of them), the A / B
// fragments of the 16x16x4 MFMA: lane (i = l & 15, q = l >> 4) supplies
// client 16a + i (A) / 16b + i (B) at columns 16q + m of MFMA m, centred by
// the stage's column mean, so 16 MFMAs cover the stage.  Stage sums are fp32
// (MFMA accumulation: an fmaf chain over 64 columns) and are added into fp64
// per stage.  Partials go to the workspace [g][tile][16 x 16]; the finish
// kernels sum them over g in a fixed order into the K x K Gram M (fp64) and
// form D = max(0, M_ii + M_jj - 2 M_ij).
//
// Accuracy: each centred value is one fp32 rounding of x - r, each stage's
// Gram entry an fp32 fmaf chain over 64 products (~1e-7 relative to
// sum |c_i c_j|), so |D - D_exact| is ~1e-7 * (|c_i|^2 + |c_j|^2): the same
// order as the reference's own fp32 torch.norm when the clients' spread is
// of the order of their distances (tests/test_gpu_dist_defenses.py checks
// the Krum selections and D against the exact-difference kernel).
constexpr int kGramMax = 128;          // clients the Gram kernel holds (8 groups of 16)
constexpr int kGramBlocksPerCU = 2;    // 2 x (2 stage buffers of 128 rows) = 143 KB of LDS per CU

__host__ __device__ inline int gram_groups(int K) { return (K + 15) / 16; }
__host__ __device__ inline int gram_tiles(int K) {
  const int nb = gram_groups(K);
  return nb * (nb + 1) / 2;
}

// tile index -> (a, b), row-major over the upper triangle of nb x nb
__device__ __forceinline__ int2 gram_tile(int t, int nb) {
  int a = 0;
  while (t >= nb - a) {
    t -= nb - a;
    ++a;
  }
  return int2{a, a + t};
}

typedef float f32x4v __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// The centred Gram on the bf16 matrix cores (the shipped kernel; the fp32-MFMA form
// it replaced, 5.3 ms at config 3, is recorded in NOTES.md §5c).
//
// Every centred value is split EXACTLY into three bf16 parts, c = h + m + l
// (h = bf16(c) rounded to nearest, m = bf16(c - h), l = c - h - m: each
// remainder is exact in fp32 and the last one has at most 8 significant bits,
// so it IS a bf16), and
//   c_i c_j = h_i h_j + h_i m_j + m_i h_j + m_i m_j + h_i l_j + l_i h_j + e,
//   |e| <= |m_i l_j| + |l_i m_j| + |l_i l_j| <= 2^-23 |c_i| |c_j|
// (|m| <= 2^-8 |c|, |l| <= 2^-8 |m|; tests/test_gram_split.py), the order of
// the fp32 rounding of each product on the f32 MFMA (2^-24).  bf16 x bf16
// products are exact in fp32 and the MFMA accumulates in fp32, so each Gram
// entry is a sum of exact products at fp32 accumulation, as on the f32 MFMA.
// Six v_mfma_f32_16x16x32_bf16 (16 cycles each) cover 32 columns of a tile
// where the f32 form needs eight 16x16x4 (32 cycles each): 96 against 256
// cycles, so the 3.0 ms matrix floor at config 3 drops to 1.1 ms, under the
// 1.64 ms of reading the rows once.
//
// LDS: the three planes of one stage, [plane][client][64 columns] bf16, rows
// of kSplitRB (160) bytes.  gfx950 serves a ds_read_b128 in the lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59},
// {36-43,48-51,60-63}, i.e. (rows 0-3, 12-15 at k-block q) with (rows 4-11 at
// q + 1): with 160-byte rows those 16 reads hit 16 distinct 16-byte bank
// groups for both k-steps (tools/lds_layout.py checks it); the 144-byte rows
// of the first version made every group 2-way.  The stores (ds_write_b64,
// 16 contiguous lanes = one 128-byte row) are conflict-free either way.  The
// split is done once per element when a stage is written, never per tile.
// Fragments (16x16x32, lane i = l & 15, q = l >> 4): A[row i][k = 8q + j] and
// B[k = 8q + j][col i] are both 16 bytes of row (16 g + i) at columns
// 32 ks + 8q .. + 7.  A wave's tiles are a contiguous run in row-major order,
// so consecutive tiles share their A group: its fragments are read once per run.
constexpr int kSplitFold = 4;  // stages summed in fp32 by the MFMAs before one fp64 fold
constexpr int kSplitRB = 160;  // bytes per plane row: 64 bf16 + padding

typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));

// two floats -> packed bf16 pair, round to nearest even (v_cvt_pk_bf16_f32)
[[maybe_unused]] __device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2v{a, b}, bf16x2v));
}
[[maybe_unused]] __device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
[[maybe_unused]] __device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// The split kernel's tile schedule: wave w takes the two rows of tiles w and
// NB - 1 - w of the group triangle (NB - w and w + 1 tiles: NB + 1 in all, the
// same for every wave at even NB; an odd NB's middle row goes alone).  Both
// rows' A fragments are read once per k-step, the B fragments ping-pong by
// tile, so tile j + 1's reads overlap tile j's six MFMAs, and every wave runs
// ONE code path (per-wave compile-time schedules spilled).
template <int PLANE>
__device__ __forceinline__ void split_frag(const unsigned char* fp, int grp, int ks, bf16x8v (&F)[3]) {
  const unsigned char* p = fp + grp * (16 * kSplitRB) + 64 * ks;
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) F[pl] = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4v*>(p + pl * PLANE));
}

[[maybe_unused]] __device__ __forceinline__ f32x4v split_mfma6(const bf16x8v (&A)[3], const bf16x8v (&B)[3], f32x4v x) {
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[0], x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[1], x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[0], x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[1], x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[2], x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], B[0], x, 0, 0, 0);
  return x;
}

// pairgram_split8_kernel: the split Gram with 8 waves per block and ONE
// block per CU, so the planes can be double-buffered (2 x 55 KB) and a stage
// needs one barrier, and each lane's raw rows are prefetched two stages
// ahead (two register sets; 16 rows per wave).  Iteration k: split stage
// k + 1 into the free plane buffer (its column sums were published before
// the last barrier), issue stage k + 3's loads into the freed registers,
// compute stage k, publish stage k + 2's column sums, barrier.  A stage's
// loads have two iterations to land.  Tiles: the row pair p (rows p and
// NB - 1 - p, as the 4-wave kernel) is shared by waves p and p + 4, which sit
// on the same SIMD: wave p takes its first ceil(n / 2) tiles, wave p + 4 the
// rest, so every SIMD runs one pair's MFMAs per stage.
constexpr int kSplit8BS = 512;

// K = 113..128 (8 groups): the 36 tiles as 2 x 2 group blocks, so one read
// of a group's fragments feeds two tiles.  Wave s (s < 4) takes a full block
// (4 tiles: rows {A0, A1} x columns {B0, B1}); wave s + 4, on the same SIMD,
// a diagonal block (3 tiles) and half of a full block (2 tiles, one column):
// 9 tiles per SIMD, 27 fragment reads per SIMD and k-step where the row-run
// schedule needs 36.
constexpr int kBlk8[8][2][5] = {
    // {A0, A1, B0, B1, diag} x 2 blocks (A0 < 0: none)
    {{0, 1, 2, 3, 0}, {-1, -1, -1, -1, 0}}, {{0, 1, 4, 5, 0}, {-1, -1, -1, -1, 0}},
    {{0, 1, 6, 7, 0}, {-1, -1, -1, -1, 0}}, {{2, 3, 4, 5, 0}, {-1, -1, -1, -1, 0}},
    {{0, 1, 0, 1, 1}, {2, 3, 6, -1, 0}},    {{2, 3, 2, 3, 1}, {2, 3, 7, -1, 0}},
    {{4, 5, 4, 5, 1}, {4, 5, 6, -1, 0}},    {{6, 7, 6, 7, 1}, {4, 5, 7, -1, 0}}};
// the (row, column) group of each accumulator slot, in gblock's order
__constant__ constexpr int kBlk8Tile[8][5][2] = {
    {{0, 2}, {0, 3}, {1, 2}, {1, 3}, {-1, -1}}, {{0, 4}, {0, 5}, {1, 4}, {1, 5}, {-1, -1}},
    {{0, 6}, {0, 7}, {1, 6}, {1, 7}, {-1, -1}}, {{2, 4}, {2, 5}, {3, 4}, {3, 5}, {-1, -1}},
    {{0, 0}, {0, 1}, {1, 1}, {2, 6}, {3, 6}},   {{2, 2}, {2, 3}, {3, 3}, {2, 7}, {3, 7}},
    {{4, 4}, {4, 5}, {5, 5}, {4, 6}, {5, 6}},   {{6, 6}, {6, 7}, {7, 7}, {4, 7}, {5, 7}}};

// one block's tiles for k-step ks: (A0,B0), (A0,B1), (A1,B0) unless diagonal,
// (A1,B1), into acc[S0 ..]; a diagonal block reads its rows once (B = A)
template <int PLANE, int A0, int A1, int B0, int B1, bool DIAG, int S0, int TPW>
__device__ __forceinline__ void gblock(const unsigned char* fp, int ks, f32x4v (&acc)[TPW]) {
  bf16x8v FA0[3], FA1[3], FB0[3], FB1[3];
  split_frag<PLANE>(fp, A0, ks, FA0);
  split_frag<PLANE>(fp, A1, ks, FA1);
  if constexpr (!DIAG) {
    split_frag<PLANE>(fp, B0, ks, FB0);
    if constexpr (B1 >= 0) split_frag<PLANE>(fp, B1, ks, FB1);
  }
  const bf16x8v(&b0)[3] = DIAG ? FA0 : FB0;
  const bf16x8v(&b1)[3] = DIAG ? FA1 : FB1;
  constexpr int s1 = S0 + 1, s2 = S0 + (B1 >= 0 ? 2 : 1), s3 = s2 + (DIAG ? 0 : 1);
  acc[S0] = split_mfma6(FA0, b0, acc[S0]);
  if constexpr (B1 >= 0) acc[s1] = split_mfma6(FA0, b1, acc[s1]);
  if constexpr (!DIAG) acc[s2] = split_mfma6(FA1, b0, acc[s2]);
  if constexpr (B1 >= 0) acc[s3] = split_mfma6(FA1, b1, acc[s3]);
}

template <int PLANE, int W, int TPW>
__device__ __forceinline__ void gblocks8(const unsigned char* fp, f32x4v (&acc)[TPW]) {
  constexpr int d0 = kBlk8[W][0][4], d1 = kBlk8[W][1][4];
  constexpr int n0 = d0 ? 3 : (kBlk8[W][0][3] >= 0 ? 4 : 2);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    gblock<PLANE, kBlk8[W][0][0], kBlk8[W][0][1], kBlk8[W][0][2], kBlk8[W][0][3], d0 != 0, 0, TPW>(fp, ks, acc);
    if constexpr (kBlk8[W][1][0] >= 0)
      gblock<PLANE, kBlk8[W][1][0], kBlk8[W][1][1], kBlk8[W][1][2], kBlk8[W][1][3], d1 != 0, n0, TPW>(fp, ks, acc);
  }
}

template <int NB>
__global__ __launch_bounds__(kSplit8BS, 1) void pairgram_split8_kernel(const float* const* __restrict__ src, int K,
                                                                     const int64_t* __restrict__ chunks,
                                                                     int64_t n_chunks, int G,
                                                                     double* __restrict__ partial) {
  constexpr int ROWS = NB * 16;
  constexpr int NT = NB * (NB + 1) / 2;
  constexpr int TPW = (NB + 2) / 2;  // ceil((NB + 1) / 2) tiles per wave, at most
  constexpr int RPW = ROWS / 8;      // staged rows per wave
  constexpr int LPW = (RPW + 3) / 4; // 16-byte loads per lane and stage (4 rows per wave-load)
  constexpr int PLANE = ROWS * kSplitRB;
  __shared__ __attribute__((aligned(16))) unsigned char sP[2][3 * PLANE];
  __shared__ float sSum[2][8][kStage];
  const int g = blockIdx.x, t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int i16 = lane & 15, q = lane >> 4;
  const float* rowp[LPW];
  bool rlive[LPW];
#pragma unroll
  for (int u = 0; u < LPW; ++u) {
    const int lr = 4 * u + q;  // row within the wave's RPW (NB = 1, 2: RPW < 4, lanes past it idle)
    const int cl = wave * RPW + lr;
    rlive[u] = lr < RPW && cl < K;
    rowp[u] = src[rlive[u] ? cl : 0];
  }
  // the row pair of this wave and its share of the pair's tiles
  const int p = wave & 3;
  const int pr1 = p, pr2 = NB - 1 - p;
  const int len1 = p < (NB + 1) / 2 ? NB - p : 0;  // row pr1's tiles (b = pr1 .. NB - 1)
  const int len2 = len1 && pr2 > pr1 ? p + 1 : 0;  // row pr2's tiles (b = pr2 .. NB - 1)
  const int half = (len1 + len2 + 1) / 2;
  const int first = wave < 4 ? 0 : half;                    // this wave's tiles: pair tiles first .. first + nmine - 1
  const int nmine = wave < 4 ? half : len1 + len2 - half;
  // as (row, first column group, count) runs: at most two
  const int r1 = first < len1 ? pr1 : pr2;
  const int b1 = first < len1 ? pr1 + first : pr2 + (first - len1);
  const int n1 = first < len1 ? (len1 - first < nmine ? len1 - first : nmine) : nmine;
  const int r2 = pr2, b2 = pr2 + (first + n1 - len1 > 0 ? first + n1 - len1 : 0);
  const int n2 = nmine - n1;
  double acc64[TPW][4];
  f32x4v acc[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    acc[j] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) acc64[j][r] = 0.0;
  }
  const float invK = 1.0f / float(K);
  int64_t c = g;
  int s0 = 0;
  f32x4 v[2][LPW];
  auto fetch = [&](f32x4 (&vv)[LPW]) __attribute__((always_inline)) {
    if (c >= n_chunks) return false;
    const int len = int(chunks[2 * c + 1]);
    const int64_t col0 = chunks[2 * c] + s0;
    const int w = len - s0 < kStage ? len - s0 : kStage;
    const int c4 = 4 * i16;
    if (w == kStage) {
#pragma unroll
      for (int u = 0; u < LPW; ++u) vv[u] = ld4<true>(rowp[u] + col0 + c4);
    } else {
#pragma unroll
      for (int u = 0; u < LPW; ++u) {
        const float* pp = rowp[u] + col0;
        const bool ok = rlive[u];
        vv[u].x = ok && c4 < w ? gptr(pp)[c4] : 0.f;
        vv[u].y = ok && c4 + 1 < w ? gptr(pp)[c4 + 1] : 0.f;
        vv[u].z = ok && c4 + 2 < w ? gptr(pp)[c4 + 2] : 0.f;
        vv[u].w = ok && c4 + 3 < w ? gptr(pp)[c4 + 3] : 0.f;
      }
    }
    s0 += kStage;
    if (s0 >= len) {
      s0 = 0;
      c += G;
    }
    return true;
  };
  auto masked = [&](const f32x4& x, int u) __attribute__((always_inline)) {
    const uint32_t m = rlive[u] ? 0xffffffffu : 0u;
    return f32x4{__uint_as_float(__float_as_uint(x.x) & m), __uint_as_float(__float_as_uint(x.y) & m),
                 __uint_as_float(__float_as_uint(x.z) & m), __uint_as_float(__float_as_uint(x.w) & m)};
  };
  auto stage_sums = [&](const f32x4 (&vv)[LPW], int sb) __attribute__((always_inline)) {
    f32x4 cs = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < LPW; ++u) cs += masked(vv[u], u);
#pragma unroll
    for (int m = 16; m <= 32; m <<= 1) {
      cs.x += __shfl_xor(cs.x, m, 64);
      cs.y += __shfl_xor(cs.y, m, 64);
      cs.z += __shfl_xor(cs.z, m, 64);
      cs.w += __shfl_xor(cs.w, m, 64);
    }
    if (q == 0) *reinterpret_cast<f32x4*>(&sSum[sb][wave][4 * i16]) = cs;
  };
  auto stage_split = [&](const f32x4 (&vv)[LPW], int sb, unsigned char* P) __attribute__((always_inline)) {
    f32x4 r = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      f32x4 s8[8];
#pragma unroll
      for (int w = 0; w < 8; ++w) s8[w] = *reinterpret_cast<const f32x4*>(&sSum[sb][w][4 * i16]);
      r = (((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]))) * invK;
    }
#pragma unroll
    for (int u = 0; u < LPW; ++u) {
      if (4 * u + q < RPW) {
        const f32x4 cc = masked(vv[u], u) - r;
        const uint32_t h01 = pk_bf16(cc.x, cc.y), h23 = pk_bf16(cc.z, cc.w);
        const float e0 = cc.x - bf16_lo(h01), e1 = cc.y - bf16_hi(h01);
        const float e2 = cc.z - bf16_lo(h23), e3 = cc.w - bf16_hi(h23);
        const uint32_t m01 = pk_bf16(e0, e1), m23 = pk_bf16(e2, e3);
        const uint32_t l01 = pk_bf16(e0 - bf16_lo(m01), e1 - bf16_hi(m01));
        const uint32_t l23 = pk_bf16(e2 - bf16_lo(m23), e3 - bf16_hi(m23));
        unsigned char* d = P + (wave * RPW + 4 * u + q) * kSplitRB + 8 * i16;
        *reinterpret_cast<u32x2v*>(d) = u32x2v{h01, h23};
        *reinterpret_cast<u32x2v*>(d + PLANE) = u32x2v{m01, m23};
        *reinterpret_cast<u32x2v*>(d + 2 * PLANE) = u32x2v{l01, l23};
      }
    }
  };
  int unfolded = 0;
  auto fold = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      // 16 wait states between the last MFMA writing acc[j] and this VALU
      // read: the compiler once left only 3 where the fold follows the MFMA
      // chain directly (NB = 1: wrong sums on the box); tools/mfma_hazards.py
      // checks every shipped build
      asm volatile("s_nop 15" : "+v"(acc[j]));
      acc64[j][0] += double(acc[j].x);
      acc64[j][1] += double(acc[j].y);
      acc64[j][2] += double(acc[j].z);
      acc64[j][3] += double(acc[j].w);
      acc[j] = f32x4v{0.f, 0.f, 0.f, 0.f};
    }
    unfolded = 0;
  };
  const int fo = i16 * kSplitRB + 16 * q;
  auto compute = [&](const unsigned char* P) __attribute__((always_inline)) {
    if constexpr (NB == 8) {
      const unsigned char* fp = P + fo;
      switch (wave) {
        case 0: gblocks8<PLANE, 0>(fp, acc); break;
        case 1: gblocks8<PLANE, 1>(fp, acc); break;
        case 2: gblocks8<PLANE, 2>(fp, acc); break;
        case 3: gblocks8<PLANE, 3>(fp, acc); break;
        case 4: gblocks8<PLANE, 4>(fp, acc); break;
        case 5: gblocks8<PLANE, 5>(fp, acc); break;
        case 6: gblocks8<PLANE, 6>(fp, acc); break;
        default: gblocks8<PLANE, 7>(fp, acc); break;
      }
      if (++unfolded == kSplitFold) fold();
      return;
    }
    if (nmine > 0) {
      const unsigned char* fp = P + fo;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8v A1[3], A2[3], B[2][3];
        split_frag<PLANE>(fp, r1, ks, A1);
        split_frag<PLANE>(fp, b1, ks, B[0]);
        if (n2) split_frag<PLANE>(fp, r2, ks, A2);
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          if (j < nmine) {
            if (j + 1 < nmine)
              split_frag<PLANE>(fp, j + 1 < n1 ? b1 + j + 1 : b2 + (j + 1 - n1), ks, B[(j + 1) & 1]);
            acc[j] = j < n1 ? split_mfma6(A1, B[j & 1], acc[j]) : split_mfma6(A2, B[j & 1], acc[j]);
          }
        }
      }
    }
    if (++unfolded == kSplitFold) fold();
  };
  // prologue: stages 0 and 1 loaded, stage 0 split, stage 1's sums published
  bool h0 = fetch(v[0]);
  bool h1 = h0 && fetch(v[1]);
  if (h0) {
    stage_sums(v[0], 0);
    lds_barrier();
    stage_split(v[0], 0, sP[0]);
    bool h2 = h1 && fetch(v[0]);  // stage 2
    if (h1) stage_sums(v[1], 1);
    lds_barrier();
    // iteration k (two at a time, so the register sets are static)
    auto iter = [&](auto cur_tag, bool& hn, bool& hnn) __attribute__((always_inline)) {
      constexpr int C = decltype(cur_tag)::value;  // k % 2
      // hn: stage k + 1 exists (in v[C ^ 1], sums in sSum[C ^ 1]); hnn: stage k + 2 (in v[C])
      bool hnnn = false;
      if (hn) {
        stage_split(v[C ^ 1], C ^ 1, sP[C ^ 1]);
        hnnn = hnn && fetch(v[C ^ 1]);  // stage k + 3
      }
      compute(sP[C]);
      if (hnn) stage_sums(v[C], C);
      lds_barrier();
      const bool more = hn;
      hn = hnn;
      hnn = hnnn;
      return more;
    };
    bool hn = h1, hnn = h2;
    while (true) {
      if (!iter(std::integral_constant<int, 0>{}, hn, hnn)) break;
      if (!iter(std::integral_constant<int, 1>{}, hn, hnn)) break;
    }
  }
  if (unfolded) fold();
  const int nout = NB == 8 ? (wave < 4 ? 4 : 5) : nmine;
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    if (j < nout) {
      int a = j < n1 ? r1 : r2, b = j < n1 ? b1 + j : b2 + (j - n1);
      if constexpr (NB == 8) {
        a = kBlk8Tile[wave][j][0];
        b = kBlk8Tile[wave][j][1];
      }
      const int tt = a * NB - a * (a - 1) / 2 + (b - a);
      double* out = partial + (int64_t(g) * NT + tt) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(4 * q + r) * 16 + i16] = acc64[j][r];
    }
  }
}


// M (K x K, fp64, both triangles) = the tiles' partials summed over the chunk
// groups in four fixed-order quarters (as tri_finish_kernel)
__global__ __launch_bounds__(256) void gram_sum_kernel(const double* __restrict__ partial, int G, int K,
                                                       double* __restrict__ M) {
  __shared__ double quarter[4][64];
  const int nb = gram_groups(K), NT = nb * (nb + 1) / 2, E = NT * 256;
  const int lane = threadIdx.x & 63, qq = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  const int ec = e < E ? e : E - 1;
  const double* p = partial + ec;
  double s[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int gg = qq;
  for (; gg + 28 < G; gg += 32) {
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += p[int64_t(gg + 4 * u) * E];
  }
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (gg + 4 * u < G) s[u] += p[int64_t(gg + 4 * u) * E];
  quarter[qq][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (qq != 0 || e >= E) return;
  const double v = (quarter[0][lane] + quarter[1][lane]) + (quarter[2][lane] + quarter[3][lane]);
  const int2 ab = gram_tile(e >> 8, nb);
  const int row = 16 * ab.x + ((e >> 4) & 15), col = 16 * ab.y + (e & 15);
  if (row >= K || col >= K) return;
  M[int64_t(row) * K + col] = v;  // a diagonal tile writes both orders itself (the same fp32 chains)
  if (ab.x != ab.y) M[int64_t(col) * K + row] = v;
}

// D[i][j] = max(0, M_ii + M_jj - 2 M_ij), 0 on the diagonal
__global__ __launch_bounds__(256) void gram_dist_kernel(const double* __restrict__ M, int K, double* __restrict__ D) {
  const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (e >= int64_t(K) * K) return;
  const int i = int(e / K), j = int(e % K);
  // M_ij + M_ji: a diagonal tile of the split kernel computes the two in a
  // different MFMA order (h_i m_j before m_i h_j), so they may differ in the
  // last bits; the sum keeps D exactly symmetric (= 2 M_ij when M is)
  const double d = (M[int64_t(i) * K + i] + M[int64_t(j) * K + j]) - (M[e] + M[int64_t(j) * K + i]);
  // negative rounding residue clamps to 0; NaN and inf pass through, so a
  // non-finite client (inf elements, or squares beyond fp32) reaches
  // gram_condition and sends "auto" to the exact kernel
  D[e] = i == j ? 0.0 : (d < 0.0 ? 0.0 : d);
}

// ---------------------------------------------------------------------------
// Clipped rebuild (norm_diff_clipping_defense.py:38-54): y = (x - r) / c + r
// in fp32 with the reference's three roundings (c = fl32 of the clip divisor;
// torch divides an fp32 tensor by a Python scalar in fp32).  Same shape as
// dist2: a block owns column tiles g, g + G, ... of FEDAGG_DIST_CHUNK columns,
// the reference tile sits in registers, wave w rebuilds clients w, w + 4, ...
// An unclipped client (c == 1) skips the division: x / 1 == x exactly.
// CClip's scaled difference (cclip_defense.py:47-52), MUL = true:
// y = fl32(fl32(x - r) * s), s = fl32 of the Python score.
template <bool MUL>
__device__ __forceinline__ f32x4 clip4(f32x4 x, f32x4 r, float c, bool one) {
  f32x4 d = f32x4{x.x - r.x, x.y - r.y, x.z - r.z, x.w - r.w};
  if constexpr (MUL) return f32x4{d.x * c, d.y * c, d.z * c, d.w * c};
  if (!one) d = f32x4{d.x / c, d.y / c, d.z / c, d.w / c};
  return f32x4{d.x + r.x, d.y + r.y, d.z + r.z, d.w + r.w};
}

// one client's rebuilt chunk -> its destination row
template <bool MUL>
__device__ __forceinline__ void clip_store(float* y, const f32x4 (&x)[kLaneCols / 4], const f32x4 (&r)[kLaneCols / 4],
                                           float c, int len, int lane) {
  const bool one = c == 1.0f;
  const bool al = (reinterpret_cast<uintptr_t>(y) & 15) == 0;
#pragma unroll
  for (int u = 0; u < kLaneCols / 4; ++u) {
    const int col = lane * 4 + 256 * u;
    const f32x4 v = clip4<MUL>(x[u], r[u], c, one);
    if (al && col + 4 <= len) {
      __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(y + col));
    } else {
      if (col < len) y[col] = v.x;
      if (col + 1 < len) y[col + 1] = v.y;
      if (col + 2 < len) y[col + 2] = v.z;
      if (col + 3 < len) y[col + 3] = v.w;
    }
  }
}

// CU clients per wave and step: all their loads are issued before the first
// store, so a lane keeps CU * kLaneCols / 4 16-byte loads in flight (one
// client at a time kept only 4, and stalled on every load before storing)
template <bool MUL, int CU>
__global__ __launch_bounds__(kBS) void clip_diff_kernel(const float* const* __restrict__ src, int K,
                                                        const float* __restrict__ ref, const float* __restrict__ div,
                                                        int64_t N, float* const* __restrict__ dst, int G) {
  const int g = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t tiles = (N + FEDAGG_DIST_CHUNK - 1) / FEDAGG_DIST_CHUNK;
  for (int64_t t = g; t < tiles; t += G) {
    const int64_t start = t * FEDAGG_DIST_CHUNK;
    const int len = int(N - start < FEDAGG_DIST_CHUNK ? N - start : FEDAGG_DIST_CHUNK);
    f32x4 r[kLaneCols / 4];
    load_chunk<false>(ref + start, len, lane, r);
    int i = w;
    for (; i + kWaves * (CU - 1) < K; i += kWaves * CU) {
      f32x4 x[CU][kLaneCols / 4];
#pragma unroll
      for (int j = 0; j < CU; ++j) load_chunk(src[i + kWaves * j] + start, len, lane, x[j]);
#pragma unroll
      for (int j = 0; j < CU; ++j)
        clip_store<MUL>(dst[i + kWaves * j] + start, x[j], r, div[i + kWaves * j], len, lane);
    }
    for (; i < K; i += kWaves) {  // the last < CU clients of this wave
      f32x4 x[kLaneCols / 4];
      load_chunk(src[i] + start, len, lane, x);
      clip_store<MUL>(dst[i] + start, x, r, div[i], len, lane);
    }
  }
}

constexpr int kClipClients = 2;  // clients in flight per wave in clip_diff_kernel

int grid_groups(int per_group_blocks, int64_t n_chunks, int64_t work_len, int64_t per_group_work) {
  int64_t G = (4096 + per_group_blocks - 1) / per_group_blocks;
  if (G > n_chunks) G = n_chunks;
  if (per_group_work > 0 && G > work_len / per_group_work) G = work_len / per_group_work;
  if (G > 65535) G = 65535;
  return int(G < 1 ? 1 : G);
}

int pair_tiles(int K) { const int T = (K + kPT - 1) / kPT; return T * (T + 1) / 2; }

template <bool MUL>
int launch_diff(const char* what, const float* const* d_src, int32_t K, const float* d_ref, const float* d_c, int64_t N,
                float* const* d_dst, fedagg_stream_t stream) {
  if (K < 1 || N < 0) return rset(FEDAGG_EINVAL, std::string(what) + ": K must be >= 1 and N >= 0");
  if (!d_src || !d_ref || !d_c || !d_dst) return rset(FEDAGG_EINVAL, std::string(what) + ": null pointer");
  if (N == 0) return FEDAGG_OK;
  const int G = grid_groups(2, (N + FEDAGG_DIST_CHUNK - 1) / FEDAGG_DIST_CHUNK, 0, 0);
  hipLaunchKernelGGL((clip_diff_kernel<MUL, kClipClients>), dim3(unsigned(G)), dim3(kBS), 0,
                     static_cast<hipStream_t>(stream), d_src, K, d_ref, d_c, N, d_dst, G);
  return rcheck(what);
}

}  // namespace

extern "C" {

int64_t fedagg_robust_work_len(int32_t kind, int32_t K, int64_t n_chunks) {
  if (K < 1 || n_chunks < 0) return -1;
  if (n_chunks == 0) return 0;
  // dist2: 1,024 blocks, the kernel's residency (4 waves per SIMD): every
  // block streams its column ranges from start to end with no second round
  // of blocks (2,048: 2.31 ms at config 3, 1,024: 2.22 ms)
  if (kind == FEDAGG_WORK_DIST2) return int64_t(K) * grid_groups(4, n_chunks, 0, 0);
  if (kind == FEDAGG_WORK_PAIRGRAM) {
    if (K > kGramMax) return -1;
    const int G = grid_groups(4096 / (256 * kGramBlocksPerCU), n_chunks, 0, 0);
    return int64_t(G) * gram_tiles(K) * 256 + int64_t(K) * K;
  }
  if (kind == FEDAGG_WORK_PAIRDIST2) {
    if (K <= kTriMax) return int64_t(16) * tri_blocks(K) * grid_groups(4, n_chunks, 0, 0);
    const int NT = pair_tiles(K);
    return int64_t(NT) * grid_groups(NT, n_chunks, 0, 0) * (kPT * kPT);
  }
  return -1;
}

int fedagg_dist2_f32(const float* const* d_src, int32_t K, const float* d_ref, const int64_t* d_chunks,
                     int64_t n_chunks, double* d_out, double* d_work, int64_t work_len, fedagg_stream_t stream) {
  if (K < 1 || n_chunks < 0) return rset(FEDAGG_EINVAL, "fedagg_dist2_f32: K must be >= 1 and n_chunks >= 0");
  if (!d_src || !d_out || (n_chunks > 0 && (!d_chunks || !d_work)))
    return rset(FEDAGG_EINVAL, "fedagg_dist2_f32: null pointer");
  auto st = static_cast<hipStream_t>(stream);
  if (n_chunks == 0) {
    if (hipMemsetAsync(d_out, 0, sizeof(double) * K, st) != hipSuccess) return rcheck("fedagg_dist2_f32");
    return FEDAGG_OK;
  }
  if (work_len < K) return rset(FEDAGG_EINVAL, "fedagg_dist2_f32: workspace smaller than K doubles");
  const int G = grid_groups(4, n_chunks, work_len, K);
  hipLaunchKernelGGL(dist2_kernel, dim3(unsigned(G)), dim3(kBS), 0, st, d_src, K, d_ref, d_chunks, n_chunks, G,
                     d_work);
  hipLaunchKernelGGL(sum_rows_kernel, dim3(unsigned(K)), dim3(256), 0, st, d_work, G, d_out);
  return rcheck("fedagg_dist2_f32");
}

int fedagg_pairdist2_f32(const float* const* d_src, int32_t K, const int64_t* d_chunks, int64_t n_chunks,
                         double* d_out, double* d_work, int64_t work_len, fedagg_stream_t stream) {
  if (K < 1 || n_chunks < 0) return rset(FEDAGG_EINVAL, "fedagg_pairdist2_f32: K must be >= 1 and n_chunks >= 0");
  if (!d_src || !d_out || (n_chunks > 0 && (!d_chunks || !d_work)))
    return rset(FEDAGG_EINVAL, "fedagg_pairdist2_f32: null pointer");
  auto st = static_cast<hipStream_t>(stream);
  if (n_chunks == 0) {
    if (hipMemsetAsync(d_out, 0, sizeof(double) * K * K, st) != hipSuccess) return rcheck("fedagg_pairdist2_f32");
    return FEDAGG_OK;
  }
  if (K <= kTriMax) {  // the whole triangle in one block per chunk group
    const int64_t per = int64_t(16) * tri_blocks(K);
    if (work_len < per) return rset(FEDAGG_EINVAL, "fedagg_pairdist2_f32: workspace too small (fedagg_robust_work_len)");
    const int G = grid_groups(4, n_chunks, work_len, per);
    if (K <= 64)
      hipLaunchKernelGGL(pairtri_kernel<16>, dim3(unsigned(G)), dim3(unsigned(tri_threads(K))), 0, st, d_src, K,
                         d_chunks, n_chunks, G, d_work);
    else
      hipLaunchKernelGGL(pairtri_kernel<32>, dim3(unsigned(G)), dim3(unsigned(tri_threads(K))), 0, st, d_src, K,
                         d_chunks, n_chunks, G, d_work);
    hipLaunchKernelGGL(tri_finish_kernel, dim3(unsigned((per + 63) / 64)), dim3(256), 0, st, d_work, G, K, d_out);
    return rcheck("fedagg_pairdist2_f32");
  }
  const int NT = pair_tiles(K);
  if (work_len < int64_t(NT) * kPT * kPT)
    return rset(FEDAGG_EINVAL, "fedagg_pairdist2_f32: workspace too small (fedagg_robust_work_len)");
  const int G = grid_groups(NT, n_chunks, work_len, int64_t(NT) * kPT * kPT);
  hipLaunchKernelGGL(pairdist_kernel, dim3(unsigned(NT), unsigned(G)), dim3(kBS), 0, st, d_src, K, d_chunks, n_chunks,
                     G, d_work);
  hipLaunchKernelGGL(pair_finish_kernel, dim3(unsigned(kPT * kPT / 64), unsigned(NT)), dim3(256), 0, st, d_work, G,
                     K, d_out);
  return rcheck("fedagg_pairdist2_f32");
}

int fedagg_pairgram2_f32(const float* const* d_src, int32_t K, const int64_t* d_chunks, int64_t n_chunks,
                         double* d_out, double* d_work, int64_t work_len, fedagg_stream_t stream) {
  if (K < 1 || K > kGramMax || n_chunks < 0)
    return rset(FEDAGG_EINVAL, "fedagg_pairgram2_f32: K must be in [1, 128] and n_chunks >= 0");
  if (!d_src || !d_out || (n_chunks > 0 && (!d_chunks || !d_work)))
    return rset(FEDAGG_EINVAL, "fedagg_pairgram2_f32: null pointer");
  auto st = static_cast<hipStream_t>(stream);
  if (n_chunks == 0) {
    if (hipMemsetAsync(d_out, 0, sizeof(double) * K * K, st) != hipSuccess) return rcheck("fedagg_pairgram2_f32");
    return FEDAGG_OK;
  }
  const int64_t per = int64_t(gram_tiles(K)) * 256;
  const int64_t mat = int64_t(K) * K;
  if (work_len < per + mat)
    return rset(FEDAGG_EINVAL, "fedagg_pairgram2_f32: workspace too small (fedagg_robust_work_len)");
  int G = grid_groups(4096 / (256 * kGramBlocksPerCU), n_chunks, work_len - mat, per);
  double* M = d_work + int64_t(G) * per;
  {
    auto kern = pairgram_split8_kernel<8>;
    switch (gram_groups(K)) {
      case 1: kern = pairgram_split8_kernel<1>; break;
      case 2: kern = pairgram_split8_kernel<2>; break;
      case 3: kern = pairgram_split8_kernel<3>; break;
      case 4: kern = pairgram_split8_kernel<4>; break;
      case 5: kern = pairgram_split8_kernel<5>; break;
      case 6: kern = pairgram_split8_kernel<6>; break;
      case 7: kern = pairgram_split8_kernel<7>; break;
      default: break;
    }
    const int G1 = G < 256 ? G : 256;  // one block per CU
    hipLaunchKernelGGL(kern, dim3(unsigned(G1)), dim3(kSplit8BS), 0, st, d_src, K, d_chunks, n_chunks, G1, d_work);
    G = G1;
  }
  hipLaunchKernelGGL(gram_sum_kernel, dim3(unsigned((per + 63) / 64)), dim3(256), 0, st, d_work, G, K, M);
  hipLaunchKernelGGL(gram_dist_kernel, dim3(unsigned((mat + 255) / 256)), dim3(256), 0, st, M, K, d_out);
  return rcheck("fedagg_pairgram2_f32");
}

int fedagg_clip_diff_f32(const float* const* d_src, int32_t K, const float* d_ref, const float* d_div, int64_t N,
                         float* const* d_dst, fedagg_stream_t stream) {
  return launch_diff<false>("fedagg_clip_diff_f32", d_src, K, d_ref, d_div, N, d_dst, stream);
}

int fedagg_scale_diff_f32(const float* const* d_src, int32_t K, const float* d_ref, const float* d_scale, int64_t N,
                          float* const* d_dst, fedagg_stream_t stream) {
  return launch_diff<true>("fedagg_scale_diff_f32", d_src, K, d_ref, d_scale, N, d_dst, stream);
}

}  // extern "C"
