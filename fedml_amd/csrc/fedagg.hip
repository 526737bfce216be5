// fedagg.hip — gfx950 (MI355X, CDNA4) kernels for server-side federated
// aggregation, exported through the C ABI declared in include/fedagg.h.
//
// What this replaces: the per-key, per-client PyTorch-eager loop of FedML's
// FedAvg reduction, python/fedml/ml/aggregator/agg_operator.py:35-44
//
//     for k in keys: for i in clients: avg[k] (=|+=) p_i[k] * (n_i / sum n)
//
// which costs 2*K*#keys eager dispatches and ~5x the algorithmic DRAM traffic
// on the CPU.  Here one launch streams every client exactly once.
//
// Design (bandwidth-bound, ~0.25 flop/B: no MFMA, no LDS round trip needed):
//   * a workgroup owns a contiguous slice of the parameter axis and walks the
//     client axis in reference order, holding the running sum in registers;
//   * 16-byte loads per lane (1 KiB per wave-instruction), U clients x V packs
//     issued back to back so every lane keeps U*V loads in flight;
//   * the per-client weight and source pointer are wave-uniform and arrive by
//     scalar loads (s_load), so the VALU only does the mul and the add;
//   * compiled with -ffp-contract=off: the mul and the add are two IEEE
//     roundings exactly like torch's `p * w` followed by `acc += t`, so fp32
//     results are bit-identical to the reference;
//   * the last workgroup of a tensor (ragged tail, or unaligned pointers) takes
//     a scalar path with identical arithmetic.
//
// Numeric conventions follow torch's CPU kernels (verified bitwise against
// golden vectors produced by the reference itself, tests/golden/):
//   fp32 * python-float : fl32(x * fl32(w))
//   bf16/f16 * float    : rnd16(fl32(f32(x) * fl32(w)))     (opmath float)
//   bf16/f16 a += b     : rnd16(fl32(f32(a) + f32(b)))
//   int64 * float       : fl32(fl32(x) * fl32(w))  -> float32 result
//   fp64 * float        : fl64(x * w)

#include <hip/hip_runtime.h>
#include <cmath>

#include <stdint.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <emmintrin.h>
#include <pthread.h>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/fedagg.h"

namespace {

constexpr int kBlock = 256;  // 4 waves of 64 lanes

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    return set_error(static_cast<int>(e),
                     std::string(what) + ": " + hipGetErrorString(e));
  }
  return FEDAGG_OK;
}

// ---------------------------------------------------------------------------
// 16-bit float helpers (round-to-nearest-even, NaN kept a quiet NaN as torch's
// c10::BFloat16 / c10::Half do).

__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(static_cast<uint32_t>(h) << 16);
}

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;  // c10 canonical NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

// Round an fp32 value to bf16 and back with gfx950's v_cvt_pk_bf16_f32 (RNE
// under the default float mode; a NaN stays a NaN).  Used for the per-client
// roundings of the reference chain; the final store uses f32_to_bf16 so a NaN
// result carries torch's canonical 0x7FC0 pattern.  The value goes into the
// HIGH half with +0 in the low half, so the packed register IS the rounded
// fp32 value: one v_cvt_pk_bf16_f32 v, 0, f per rounding, where converting
// into the low half needs a shift or mask per value afterwards (1.5
// instructions per rounding; the chain has two per client and element).
typedef float fedagg_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 fedagg_b2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float bf16_round(float f) {
  const fedagg_b2 b = __builtin_convertvector((fedagg_f2){0.0f, f}, fedagg_b2);
  return __builtin_bit_cast(float, b);
}

__device__ __forceinline__ float f16_to_f32(uint16_t h) {
  _Float16 v;
  __builtin_memcpy(&v, &h, 2);
  return static_cast<float>(v);
}

__device__ __forceinline__ uint16_t f32_to_f16(float f) {
  _Float16 v = static_cast<_Float16>(f);  // v_cvt_f16_f32: RNE
  uint16_t h;
  __builtin_memcpy(&h, &v, 2);
  return h;
}

// ---------------------------------------------------------------------------
// Reduction operators.  Each defines the storage types, the weight type, and
// the two steps of the reference chain: first() for client 0 (the `=` branch,
// agg_operator.py:41-42) and step() for the others (the `+=` branch, :43-44).

struct OpF32 {  // fp32 FedAvg
  using in_t = float; using out_t = float; using acc_t = float; using w_t = float;
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return x * w; }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return a + x * w; }
  static __device__ __forceinline__ out_t fin(acc_t a) { return a; }
};

struct OpBF16Ref {  // bf16, torch CPU chain (round after every op)
  using in_t = uint16_t; using out_t = uint16_t; using acc_t = float; using w_t = float;
  static __device__ __forceinline__ float r(float f) { return bf16_round(f); }
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return r(bf16_to_f32(x) * w); }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return r(a + r(bf16_to_f32(x) * w)); }
  // two neighbouring elements, the same arithmetic element by element: the
  // mul and the add as v_pk_mul_f32 / v_pk_add_f32 (each lane-half IEEE RNE,
  // as the scalar ops), the four roundings one v_cvt_pk_bf16_f32 each
  static __device__ __forceinline__ void step2(acc_t& a0, acc_t& a1, in_t x0, in_t x1, w_t w) {
    fedagg_f2 p = (fedagg_f2){bf16_to_f32(x0), bf16_to_f32(x1)} * (fedagg_f2){w, w};
    p = (fedagg_f2){r(p.x), r(p.y)};
    const fedagg_f2 t = (fedagg_f2){a0, a1} + p;
    a0 = r(t.x);
    a1 = r(t.y);
  }
  static __device__ __forceinline__ out_t fin(acc_t a) { return f32_to_bf16(a); }
};

struct OpBF16Acc32 {  // bf16 in, fp32 accumulate, one rounding at the end
  using in_t = uint16_t; using out_t = uint16_t; using acc_t = float; using w_t = float;
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return bf16_to_f32(x) * w; }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return a + bf16_to_f32(x) * w; }
  static __device__ __forceinline__ out_t fin(acc_t a) { return f32_to_bf16(a); }
};

struct OpBF16F32Out {  // bf16 in, fp32 partial out (multi-GPU pre-reduction)
  using in_t = uint16_t; using out_t = float; using acc_t = float; using w_t = float;
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return bf16_to_f32(x) * w; }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return a + bf16_to_f32(x) * w; }
  static __device__ __forceinline__ out_t fin(acc_t a) { return a; }
};

// f16, torch CPU chain.  torch rounds x * w to fp32 and then to f16 (two
// roundings); left alone, the compiler folds mul + f16 rounding into one
// v_fma_mixlo_f16, which rounds the exact product once and differs in rare
// near-tie cases (1 element in 255 at K = 600).  The product is made opaque
// so it is materialised in fp32 first.  (a + b of two f16 values is exact in
// fp32 up to the final rounding, so v_add_f16 there is the same chain.)
__device__ __forceinline__ float fp32_materialise(float v) {
  asm("" : "+v"(v));
  return v;
}
struct OpF16Ref {
  using in_t = uint16_t; using out_t = uint16_t; using acc_t = float; using w_t = float;
  static __device__ __forceinline__ float r(float f) { return f16_to_f32(f32_to_f16(f)); }
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return r(fp32_materialise(f16_to_f32(x) * w)); }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) {
    return r(a + r(fp32_materialise(f16_to_f32(x) * w)));
  }
  static __device__ __forceinline__ out_t fin(acc_t a) { return f32_to_f16(a); }
};

struct OpF16Acc32 {
  using in_t = uint16_t; using out_t = uint16_t; using acc_t = float; using w_t = float;
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return f16_to_f32(x) * w; }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return a + f16_to_f32(x) * w; }
  static __device__ __forceinline__ out_t fin(acc_t a) { return f32_to_f16(a); }
};

struct OpF64 {
  using in_t = double; using out_t = double; using acc_t = double; using w_t = double;
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return x * w; }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return a + x * w; }
  static __device__ __forceinline__ out_t fin(acc_t a) { return a; }
};

struct OpI64F32 {  // int64 buffers (BN num_batches_tracked) promote to float32
  using in_t = int64_t; using out_t = float; using acc_t = float; using w_t = float;
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return static_cast<float>(x) * w; }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return a + static_cast<float>(x) * w; }
  static __device__ __forceinline__ out_t fin(acc_t a) { return a; }
};

// Unweighted sums (FedAvg_seq / FedDyn), source dtype preserved.
// MPI simulation FedAvg (simulation/mpi/fedavg/FedAVGAggregator.py:99-116):
// `local_model_params[k] * local_sample_number / training_num` is evaluated
// left to right, so every client's term is fl(fl(p * n_i) / N): two roundings
// (a correctly rounded division; hipcc's default) instead of the plugin
// path's fl(p * fl(n_i / N)).  The weight of client i carries (n_i, N) as the
// tensor's opmath type rounds them.
struct MulDivF { float n, d; };
struct MulDivD { double n, d; };
// int64 rows: an integral n_i multiplies in int64 (two's-complement wrap, as
// torch's int64 * int), then true division promotes to float32; a float n_i
// promotes first: fl32(fl32(v) * fl32(n_i)).
struct MulDivI { int64_t n; float nf, d; int32_t is_int, pad; };

struct OpF32MulDiv {
  using in_t = float; using out_t = float; using acc_t = float; using w_t = MulDivF;
  static __device__ __forceinline__ float term(in_t x, w_t w) { return fp32_materialise(x * w.n) / w.d; }
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return term(x, w); }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return a + term(x, w); }
  static __device__ __forceinline__ out_t fin(acc_t a) { return a; }
};
struct OpBF16MulDiv {  // torch CPU chain: bf16 after the mul, the div and the add
  using in_t = uint16_t; using out_t = uint16_t; using acc_t = float; using w_t = MulDivF;
  static __device__ __forceinline__ float r(float f) { return bf16_round(f); }
  static __device__ __forceinline__ float term(in_t x, w_t w) { return r(r(bf16_to_f32(x) * w.n) / w.d); }
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return term(x, w); }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return r(a + term(x, w)); }
  static __device__ __forceinline__ out_t fin(acc_t a) { return f32_to_bf16(a); }
};
struct OpF16MulDiv {  // fp32 results rounded to f16 after every op (products kept in fp32 first)
  using in_t = uint16_t; using out_t = uint16_t; using acc_t = float; using w_t = MulDivF;
  static __device__ __forceinline__ float r(float f) { return f16_to_f32(f32_to_f16(f)); }
  static __device__ __forceinline__ float term(in_t x, w_t w) {
    return r(fp32_materialise(r(fp32_materialise(f16_to_f32(x) * w.n)) / w.d));
  }
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return term(x, w); }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return r(a + term(x, w)); }
  static __device__ __forceinline__ out_t fin(acc_t a) { return f32_to_f16(a); }
};
struct OpF64MulDiv {
  using in_t = double; using out_t = double; using acc_t = double; using w_t = MulDivD;
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return (x * w.n) / w.d; }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return a + (x * w.n) / w.d; }
  static __device__ __forceinline__ out_t fin(acc_t a) { return a; }
};
struct OpI64MulDiv {
  using in_t = int64_t; using out_t = float; using acc_t = float; using w_t = MulDivI;
  static __device__ __forceinline__ float term(in_t x, w_t w) {
    const float v = w.is_int ? static_cast<float>(static_cast<int64_t>(static_cast<uint64_t>(x) *
                                                                      static_cast<uint64_t>(w.n)))
                             : fp32_materialise(static_cast<float>(x) * w.nf);
    return v / w.d;
  }
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return term(x, w); }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return a + term(x, w); }
  static __device__ __forceinline__ out_t fin(acc_t a) { return a; }
};

struct OpSumF32 {
  using in_t = float; using out_t = float; using acc_t = float; using w_t = float;
  static __device__ __forceinline__ acc_t first(in_t x, w_t) { return x; }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t) { return a + x; }
  static __device__ __forceinline__ out_t fin(acc_t a) { return a; }
};
struct OpSumBF16 {
  using in_t = uint16_t; using out_t = uint16_t; using acc_t = float; using w_t = float;
  static __device__ __forceinline__ acc_t first(in_t x, w_t) { return bf16_to_f32(x); }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t) { return OpBF16Ref::r(a + bf16_to_f32(x)); }
  static __device__ __forceinline__ out_t fin(acc_t a) { return f32_to_bf16(a); }
};
struct OpSumF16 {
  using in_t = uint16_t; using out_t = uint16_t; using acc_t = float; using w_t = float;
  static __device__ __forceinline__ acc_t first(in_t x, w_t) { return f16_to_f32(x); }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t) { return OpF16Ref::r(a + f16_to_f32(x)); }
  static __device__ __forceinline__ out_t fin(acc_t a) { return f32_to_f16(a); }
};
struct OpSumF64 {
  using in_t = double; using out_t = double; using acc_t = double; using w_t = float;
  static __device__ __forceinline__ acc_t first(in_t x, w_t) { return x; }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t) { return a + x; }
  static __device__ __forceinline__ out_t fin(acc_t a) { return a; }
};
struct OpSumI64 {  // two's-complement wrap, as torch's int64 add
  using in_t = int64_t; using out_t = int64_t; using acc_t = uint64_t; using w_t = float;
  static __device__ __forceinline__ acc_t first(in_t x, w_t) { return static_cast<uint64_t>(x); }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t) { return a + static_cast<uint64_t>(x); }
  static __device__ __forceinline__ out_t fin(acc_t a) { return static_cast<int64_t>(a); }
};
struct OpSumI32 {
  using in_t = int32_t; using out_t = int32_t; using acc_t = uint32_t; using w_t = float;
  static __device__ __forceinline__ acc_t first(in_t x, w_t) { return static_cast<uint32_t>(x); }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t) { return a + static_cast<uint32_t>(x); }
  static __device__ __forceinline__ out_t fin(acc_t a) { return static_cast<int32_t>(a); }
};

// Secure aggregation over a finite field (LightSecAgg, core/mpc/lightsecagg.py).
// numpy int64 semantics: adds wrap, np.mod is a floor modulo (sign of p).
__device__ __forceinline__ int64_t floor_mod(int64_t a, int64_t p) {
  int64_t r = a % p;
  if (r != 0 && ((r < 0) != (p < 0))) r += p;
  return r;
}
__device__ __forceinline__ int64_t wrap_add(int64_t a, int64_t b) {
  return static_cast<int64_t>(static_cast<uint64_t>(a) + static_cast<uint64_t>(b));
}

// aggregate_models_in_finite (:134-148): w = x_0 ; w = (w + x_i) mod p.  The
// "weight" operand carries p.  Field elements (0 <= a, b < p) take the
// conditional-subtract path; anything else the exact 64-bit floor modulo.
struct OpSumModI64 {
  using in_t = int64_t; using out_t = int64_t; using acc_t = int64_t; using w_t = int64_t;
  static __device__ __forceinline__ acc_t first(in_t x, w_t) { return x; }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t p) {
    if (p > 0 && static_cast<uint64_t>(a) < static_cast<uint64_t>(p) &&
        static_cast<uint64_t>(x) < static_cast<uint64_t>(p) && p <= (int64_t(1) << 62)) {
      const int64_t s2 = a + x;
      return s2 >= p ? s2 - p : s2;
    }
    return floor_mod(wrap_add(a, x), p);
  }
  static __device__ __forceinline__ out_t fin(acc_t a) { return a; }
};

// Plain wrapping int64 sum (the first half of aggregate_model_reconstruction).
struct OpWrapSumI64 {
  using in_t = int64_t; using out_t = int64_t; using acc_t = int64_t; using w_t = int64_t;
  static __device__ __forceinline__ acc_t first(in_t x, w_t) { return x; }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t) { return wrap_add(a, x); }
  static __device__ __forceinline__ out_t fin(acc_t a) { return a; }
};

// ---------------------------------------------------------------------------
// 16-byte packs.

template <class T, int E>
struct alignas(16) Pack {
  T v[E];
};

// Client rows arrive through pointer tables, which hipcc cannot prove are
// global memory: without the cast it issues FLAT loads, which also count on
// lgkmcnt and so get waited for together with the scalar loads of the next
// client pointers.  All device pointers here are global (hipMalloc / torch).
template <class T>
__device__ __forceinline__ const T __attribute__((address_space(1)))* as_global(const T* p) {
  return (const T __attribute__((address_space(1)))*)(p);
}

template <class T, bool NT>
__device__ __forceinline__ Pack<T, 16 / sizeof(T)> load_pack(const T* p) {
  typedef const u32x4 __attribute__((address_space(1)))* gvec;
  const gvec g = (gvec)(p);
  u32x4 r;
  if constexpr (NT) {
    r = __builtin_nontemporal_load(g);
  } else {
    r = *g;
  }
  Pack<T, 16 / sizeof(T)> o;
  __builtin_memcpy(&o, &r, 16);
  return o;
}

template <class T, int E>
__device__ __forceinline__ void store_pack(T* p, const T (&v)[E]) {
  constexpr int bytes = E * sizeof(T);
  static_assert(bytes == 32 || bytes == 16 || bytes == 8, "pack store is 8, 16 or 32 bytes");
  if constexpr (bytes == 32) {  // bf16 -> fp32 partial: two 16-byte halves
    u32x4 r0, r1;
    __builtin_memcpy(&r0, v, 16);
    __builtin_memcpy(&r1, reinterpret_cast<const char*>(v) + 16, 16);
    __builtin_nontemporal_store(r0, reinterpret_cast<u32x4*>(p));
    __builtin_nontemporal_store(r1, reinterpret_cast<u32x4*>(p) + 1);
  } else if constexpr (bytes == 16) {
    u32x4 r;
    __builtin_memcpy(&r, v, 16);
    __builtin_nontemporal_store(r, reinterpret_cast<u32x4*>(p));
  } else {
    u32x2 r;
    __builtin_memcpy(&r, v, 8);
    __builtin_nontemporal_store(r, reinterpret_cast<u32x2*>(p));
  }
}

// Per-client weight sources.  PtrW reads a device array (s_load, wave-uniform);
// InlW carries up to kInlineK weights by value in the kernel arguments, so a
// round needs no weight upload at all (FEDAGG_HOST_WEIGHTS).
template <class T>
struct PtrW {
  const T* p;
  __device__ __forceinline__ T operator[](int i) const { return p ? p[i] : T{}; }
};
template <class T>
struct ConstW {  // one value for every client (the field prime of the mod-p sum)
  T v;
  __device__ __forceinline__ T operator[](int) const { return v; }
};
constexpr int kInlineK = 256;
template <class T>
struct InlW {
  T v[kInlineK];
  __device__ __forceinline__ T operator[](int i) const { return v[i]; }
};

// One tensor ("segment") of the reduction: K source pointers and its length.
template <class OP>
struct Seg {
  const typename OP::in_t* const* src;  // device table of K pointers
  int64_t numel;
};

// Epilogues: what happens to a finished running sum.  pack() takes the E sums
// of one 16-byte input pack at element offset `off`, one() a single element.

// Plain FedAvg: round to the output dtype and store (non-temporal: written once).
template <class OP>
struct StoreEpi {
  typename OP::out_t* out;
  static constexpr int E = 16 / sizeof(typename OP::in_t);
  struct Pre {};  // nothing to prefetch
  __device__ __forceinline__ Pre pre(int64_t) const { return {}; }
  __device__ __forceinline__ void pack(int64_t off, const typename OP::acc_t (&acc)[E], const Pre&) const {
    typename OP::out_t o[E];
#pragma unroll
    for (int e = 0; e < E; ++e) o[e] = OP::fin(acc[e]);
    store_pack<typename OP::out_t, E>(out + off, o);
  }
  __device__ __forceinline__ void one(int64_t e, typename OP::acc_t a) const { out[e] = OP::fin(a); }
};

// FedOpt server step fused onto the fp32 average (FedOptAggregator.py:104-125
// with torch.optim.SGD): the average never goes to HBM.
//   g = p_old - avg ; buf = first ? g : fl(fl(buf*m) + g) ; p = fma(buf, -lr, p_old)
// momentum == 0: torch steps with g directly and keeps no buffer.
struct SgdEpi {
  float* p;
  float* mom;  // nullptr when momentum == 0
  float neg_lr, m;
  int first;
  static constexpr int E = 4;
  // p_old and the momentum buffer are independent of the client loop: load
  // them before it so their latency hides under the stream.
  struct Pre {
    Pack<float, 4> p, m;
  };
  __device__ __forceinline__ Pre pre(int64_t off) const {
    Pre r;
    r.p = load_pack<float, true>(p + off);
    r.m = {};
    if (mom && !first) r.m = load_pack<float, true>(mom + off);
    return r;
  }
  __device__ __forceinline__ float step1(float po, float avg, float* mb) const {
    const float g = po - avg;
    float b = g;
    if (mom) {
      if (!first) {
        const float t = *mb * m;  // buf.mul_(m)
        b = t + g;                // .add_(grad): two roundings (-ffp-contract=off)
      }
      *mb = b;
    }
    return __builtin_fmaf(b, neg_lr, po);  // p.add_(buf, alpha=-lr): torch's fused fmadd
  }
  __device__ __forceinline__ void pack(int64_t off, const float (&acc)[E], const Pre& pr) const {
    float po[E], mo[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float mb = pr.m.v[e];
      po[e] = step1(pr.p.v[e], acc[e], &mb);
      mo[e] = mb;
    }
    store_pack<float, E>(p + off, po);
    if (mom) store_pack<float, E>(mom + off, mo);
  }
  __device__ __forceinline__ void one(int64_t e, float a) const {
    float mb = (mom && !first) ? mom[e] : 0.f;
    p[e] = step1(p[e], a, &mb);
    if (mom) mom[e] = mb;
  }
};

// Fused server Adam step (sp/fedopt/fedopt_api.py:121-130 with torch.optim.Adam's
// single-tensor CPU path, amsgrad off, weight_decay 0).  Per element, with the
// host-computed fp32 scalars of fedagg_adam_scalars():
//   g = p_old - avg
//   m = lerp(m, g, w1)          torch's vectorised lerp: one fma
//   v = fma(fl(c2*g), g, fl(v*beta2))   mul_(beta2).addcmul_(g, g, value=c2)
//   p = p_old + fl(nss*m) / (fl(sqrt(v) / bc2s) + eps)   addcdiv_, no fma
//
// AdamW (decoupled weight decay, torch.optim.AdamW = Adam with
// decoupled_weight_decay) first scales the parameter, param.mul_(1 - lr*wd),
// with the gradient already set from the unscaled one:
//   p = fl(p_old * decay) + fl(nss*m) / denom,  decay = fl32(1 - lr*wd)
// decoupled == 0 (Adam) never multiplies.
struct AdamEpi {
  float* p;
  float* m;
  float* v;
  float w1, beta2, c2, bc2s, eps, nss;
  int first;  // exp_avg / exp_avg_sq are zero before torch's first step: skip their loads
  float decay = 1.0f;
  int decoupled = 0;
  static constexpr int E = 4;
  // p_old and exp_avg are prefetched before the client loop like SgdEpi's
  // operands; exp_avg_sq is loaded in the epilogue (a third prefetched pack
  // per V takes the kernel past 128 VGPRs: occupancy 3 instead of 4).
  struct Pre {
    Pack<float, 4> p, m;
  };
  __device__ __forceinline__ Pre pre(int64_t off) const {
    Pre r;
    r.p = load_pack<float, true>(p + off);
    r.m = {};
    if (!first) r.m = load_pack<float, true>(m + off);
    return r;
  }
  __device__ __forceinline__ float step1(float po, float avg, float* mm, float* vv) const {
    const float g = po - avg;
    const float d = g - *mm;
    *mm = __builtin_fabsf(w1) < 0.5f ? __builtin_fmaf(w1, d, *mm) : __builtin_fmaf(w1 - 1.0f, d, g);
    const float vb = *vv * beta2;
    *vv = __builtin_fmaf(c2 * g, g, vb);
    const float denom = __builtin_sqrtf(*vv) / bc2s + eps;
    const float pb = decoupled ? po * decay : po;
    return pb + (nss * *mm) / denom;
  }
  __device__ __forceinline__ void pack(int64_t off, const float (&acc)[E], const Pre& pr) const {
    float po[E], mo[E], vo[E];
    Pack<float, 4> vp = {};
    if (!first) vp = load_pack<float, true>(v + off);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      mo[e] = pr.m.v[e];
      vo[e] = vp.v[e];
      po[e] = step1(pr.p.v[e], acc[e], &mo[e], &vo[e]);
    }
    store_pack<float, E>(p + off, po);
    store_pack<float, E>(m + off, mo);
    store_pack<float, E>(v + off, vo);
  }
  __device__ __forceinline__ void one(int64_t e, float a) const {
    float mm = first ? 0.f : m[e];
    float vv = first ? 0.f : v[e];
    p[e] = step1(p[e], a, &mm, &vv);
    m[e] = mm;
    v[e] = vv;
  }
};

// Fused server Adagrad step (sp/fedopt/fedopt_api.py:121-130 with
// torch.optim.Adagrad's single-tensor CPU path: weight_decay 0,
// initial_accumulator_value 0 before the first step).  Per element:
//   g = p_old - avg
//   sum = fma(g, g, sum)                  addcmul_(g, g, value=1), fused
//   p = p_old + fl(neg_clr * g) / (sqrt(sum) + eps)   addcdiv_, not fused
// neg_clr = -lr / (1 + (step-1) * lr_decay) as fp32 (host side).
//
// RMSprop (torch.optim.RMSprop single-tensor CPU path, momentum 0, not
// centered, weight_decay 0) is the same step with a decaying accumulator:
//   square_avg.mul_(alpha).addcmul_(g, g, value=1-alpha)
//                                  = fma(fl(c*g), g, fl(sq*alpha)), c = fl32(1-alpha)
//   avg = fl(sqrt(square_avg) + eps);  p = p_old + fl(fl(-lr*g) / avg)
// Adagrad is a = c = 1 (fl(1*g) = g, fl(sum*1) = sum: bit-identical).
struct AdagradEpi {
  float* p;
  float* sum;
  float neg_clr, eps;
  float a = 1.0f, c = 1.0f;
  static constexpr int E = 4;
  struct Pre {
    Pack<float, 4> p, s;
  };
  __device__ __forceinline__ Pre pre(int64_t off) const {
    return {load_pack<float, true>(p + off), load_pack<float, true>(sum + off)};
  }
  __device__ __forceinline__ float step1(float po, float avg, float* ss) const {
    const float g = po - avg;
    *ss = __builtin_fmaf(c * g, g, *ss * a);
    const float std_ = __builtin_sqrtf(*ss) + eps;
    return po + (neg_clr * g) / std_;
  }
  __device__ __forceinline__ void pack(int64_t off, const float (&acc)[E], const Pre& pr) const {
    float po[E], so[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      so[e] = pr.s.v[e];
      po[e] = step1(pr.p.v[e], acc[e], &so[e]);
    }
    store_pack<float, E>(p + off, po);
    store_pack<float, E>(sum + off, so);
  }
  __device__ __forceinline__ void one(int64_t e, float a) const {
    float ss = sum[e];
    p[e] = step1(p[e], a, &ss);
    sum[e] = ss;
  }
};

// The other elementwise optimizers FedML's OptRepo can name
// (sp/fedopt/optrepo.py:10: torch.optim's direct Optimizer subclasses), each
// as FedOptAPI builds it (lr only, torch defaults; fedopt_api.py:78-85) and
// fused onto the fp32 average like AdamEpi.  Per element, following torch
// 2.10's single-tensor CPU paths op by op (one rounding per torch op, the
// fused ones as fmaf; fedagg_optrepo_scalars computes the host scalars):
//
//   Adamax   (adamax.py:265-303)   m = lerp(m, g, w1); u = max(u*b2, |g| + eps)  (NaN wins);
//                                  p = p + (s*m)/u
//   NAdam    (nadam.py:330-379)    m = lerp; v = fma(c2*g, g, v*b2); d = sqrt(v/bc2) + eps;
//                                  p = p + (s1*g)/d; p = p + (s2*m)/d
//   RAdam    (radam.py:301-360)    m, v as NAdam; x = (m/bc1)*lr; rectified steps (rho_t > 5):
//                                  x = (x * ((1/(sqrt(v) + eps)) * bc2s)) * rect; p = p - x
//   Adadelta (adadelta.py:281-302) sq = fma(c*g, g, sq*rho); d = sqrt(acc + eps) / sqrt(sq + eps) * g;
//                                  acc = fma(c*d, d, acc*rho); p = fma(d, -lr, p)
//   ASGD     (asgd.py:247-275)     p = fma(g, -eta, p*decay); ax = p (mu == 1) or ax + (p - ax)*mu
//   Rprop    (rprop.py:257-291)    f = {1.2, 0.5, 1}[sign(g*prev)]; ss = clamp(ss*f, 1e-6, 50);
//                                  g' = f == 0.5 ? 0 : g; p = fma(-sign(g'), ss, p); prev = g'
//
// state0 / state1 are the optimizer's two per-element buffers (Adamax:
// exp_avg / exp_inf; NAdam, RAdam: exp_avg / exp_avg_sq; Adadelta:
// square_avg / acc_delta; ASGD: ax / unused; Rprop: prev / step_size), in
// the state torch creates before its first step.  p_old and state0 are
// prefetched before the client loop, state1 is read in the epilogue (the
// 128-VGPR cap of reduce_fused_kernel, as for Adam).
enum : int32_t { kOptAdamax = 1, kOptNAdam = 2, kOptRAdam = 3, kOptAdadelta = 4, kOptASGD = 5, kOptRprop = 6 };

__device__ __forceinline__ float lerp_fma(float m, float g, float w) {  // torch's vectorised lerp_
  const float d = g - m;
  return __builtin_fabsf(w) < 0.5f ? __builtin_fmaf(w, d, m) : __builtin_fmaf(w - 1.0f, d, g);
}
// torch.sign: (0 < x) - (x < 0), so +0 for ±0 AND for NaN (the robust-LR sign
// sum of a column holding a NaN still counts the other clients' signs)
__device__ __forceinline__ float sign_of(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }
__device__ __forceinline__ float max_nan(float a, float b) {  // torch.maximum: a NaN operand wins
  return (a != a || b != b) ? __builtin_nanf("") : __builtin_fmaxf(a, b);
}

template <int OPT>
struct OptRepoEpi {
  float* p;
  float* s0;
  float* s1;
  float k[9];  // fedagg_optrepo_scalars' out9, per optimizer
  static constexpr int E = 4;
  static constexpr bool kS0 = OPT != kOptASGD;  // ASGD reads ax only while mu != 1
  struct Pre {
    Pack<float, 4> p, a;
  };
  __device__ __forceinline__ Pre pre(int64_t off) const {
    Pre r;
    r.p = load_pack<float, true>(p + off);
    r.a = {};
    if (kS0 || k[3] != 1.0f) r.a = load_pack<float, true>(s0 + off);
    return r;
  }
  __device__ __forceinline__ float step1(float po, float avg, float* a0, float* a1) const {
    const float g = po - avg;
    if constexpr (OPT == kOptAdamax) {
      *a0 = lerp_fma(*a0, g, k[0]);
      *a1 = max_nan(*a1 * k[1], __builtin_fabsf(g) + k[2]);
      return po + (k[3] * *a0) / *a1;
    } else if constexpr (OPT == kOptNAdam) {
      *a0 = lerp_fma(*a0, g, k[0]);
      *a1 = __builtin_fmaf(k[2] * g, g, *a1 * k[1]);
      const float d = __builtin_sqrtf(*a1 / k[3]) + k[4];
      const float p1 = po + (k[5] * g) / d;
      return p1 + (k[6] * *a0) / d;
    } else if constexpr (OPT == kOptRAdam) {
      *a0 = lerp_fma(*a0, g, k[0]);
      *a1 = __builtin_fmaf(k[2] * g, g, *a1 * k[1]);
      float x = (*a0 / k[3]) * k[4];
      if (k[5] != 0.0f) {
        const float ad = (1.0f / (__builtin_sqrtf(*a1) + k[6])) * k[7];
        x = (x * ad) * k[8];
      }
      return po - x;
    } else if constexpr (OPT == kOptAdadelta) {
      *a0 = __builtin_fmaf(k[1] * g, g, *a0 * k[0]);
      const float sd = __builtin_sqrtf(*a0 + k[2]);
      const float d = (__builtin_sqrtf(*a1 + k[2]) / sd) * g;
      *a1 = __builtin_fmaf(k[1] * d, d, *a1 * k[0]);
      return __builtin_fmaf(d, k[3], po);
    } else if constexpr (OPT == kOptASGD) {
      const float pn = __builtin_fmaf(g, k[1], po * k[0]);
      *a0 = k[3] == 1.0f ? pn : *a0 + (pn - *a0) * k[2];
      return pn;
    } else {  // kOptRprop
      const float sg = sign_of(g * *a0);
      const float f = sg > 0.f ? k[0] : (sg < 0.f ? k[1] : 1.0f);
      const float ss = *a1 * f;
      *a1 = ss != ss ? ss : __builtin_fminf(__builtin_fmaxf(ss, k[2]), k[3]);
      const float g2 = f == k[1] ? 0.0f : g;
      *a0 = g2;
      return __builtin_fmaf(-sign_of(g2), *a1, po);
    }
  }
  __device__ __forceinline__ void pack(int64_t off, const float (&acc)[E], const Pre& pr) const {
    float po[E], ao[E], bo[E];
    Pack<float, 4> b = {};
    if constexpr (OPT != kOptASGD) b = load_pack<float, true>(s1 + off);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      ao[e] = pr.a.v[e];
      bo[e] = b.v[e];
      po[e] = step1(pr.p.v[e], acc[e], &ao[e], &bo[e]);
    }
    store_pack<float, E>(p + off, po);
    store_pack<float, E>(s0 + off, ao);
    if constexpr (OPT != kOptASGD) store_pack<float, E>(s1 + off, bo);
  }
  __device__ __forceinline__ void one(int64_t e, float a) const {
    float a0 = (kS0 || k[3] != 1.0f) ? s0[e] : 0.f;
    float a1 = OPT != kOptASGD ? s1[e] : 0.f;
    p[e] = step1(p[e], a, &a0, &a1);
    s0[e] = a0;
    if constexpr (OPT != kOptASGD) s1[e] = a1;
  }
};

// LightSecAgg model reconstruction epilogue
// (cross_silo/lightsecagg/lsa_fedml_aggregator.py:139-166 with
// core/mpc/lightsecagg.py:157-182): on the wrapping int64 client sum
//   m = (sum - mask) mod p ; v = m > (p-1)/2 ? m - p : m   (my_q_inv, float64)
//   out = fl32( fl32(v / 2^q) * fl32(w) )   (torch.Tensor(...) then * (1/K))
struct LsaEpi {
  const int64_t* mask;
  float* out;
  int64_t p;
  double inv_scale;  // 2^-q (exact)
  float w;
  static constexpr int E = 2;
  struct Pre {
    Pack<int64_t, 2> m;
  };
  __device__ __forceinline__ Pre pre(int64_t off) const { return {load_pack<int64_t, true>(mask + off)}; }
  __device__ __forceinline__ float one_value(int64_t acc, int64_t mk) const {
    const int64_t m = floor_mod(wrap_add(acc, -mk), p);
    // flag = X_q - (p-1)/2 > 0, computed by numpy in float64
    const double xq = static_cast<double>(m);
    const double v = (xq - (static_cast<double>(p) - 1.0) / 2.0 > 0.0) ? xq - static_cast<double>(p) : xq;
    const float f = static_cast<float>(v * inv_scale);  // exact scale, then RNE to fp32
    return f * w;
  }
  __device__ __forceinline__ void pack(int64_t off, const int64_t (&acc)[E], const Pre& pr) const {
    float o[E];
#pragma unroll
    for (int e = 0; e < E; ++e) o[e] = one_value(acc[e], pr.m.v[e]);
    store_pack<float, E>(out + off, o);
  }
  __device__ __forceinline__ void one(int64_t e, int64_t acc) const { out[e] = one_value(acc, mask[e]); }
};

// Robust learning rate (RobustLearningRateDefense.run,
// core/security/defense/robust_learning_rate_defense.py:35-62): the FedAvg
// chain of the FedAvg branch, and in the same pass the coordinate's sum of the
// clients' torch.sign values (exact in fp32 below 2^24 clients; a NaN input
// makes it NaN, as torch.sign does); the epilogue applies
//   lr = |Σ sign|;  lr[lr < thr] = -1;  lr[lr >= thr] = 1;  out = lr * avg
// in that order (a NaN lr stays NaN), the multiply by ±1 exact.
struct RlrAcc {
  float a, s;
};
struct OpF32Rlr {
  using in_t = float; using out_t = float; using acc_t = RlrAcc; using w_t = float;
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return {x * w, sign_of(x)}; }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return {a.a + x * w, a.s + sign_of(x)}; }
};
struct RlrEpi {
  float* out;
  float thr;  // fl32(robust_threshold): torch compares the fp32 sign sum with the Python number in fp32
  static constexpr int E = 4;
  struct Pre {};
  __device__ __forceinline__ Pre pre(int64_t) const { return {}; }
  __device__ __forceinline__ float one_value(RlrAcc acc) const {
    float lr = fabsf(acc.s);
    lr = lr < thr ? -1.f : lr;
    lr = lr >= thr ? 1.f : lr;
    return lr * acc.a;
  }
  __device__ __forceinline__ void pack(int64_t off, const RlrAcc (&acc)[E], const Pre&) const {
    float o[E];
#pragma unroll
    for (int e = 0; e < E; ++e) o[e] = one_value(acc[e]);
    store_pack<float, E>(out + off, o);
  }
  __device__ __forceinline__ void one(int64_t e, RlrAcc acc) const { out[e] = one_value(acc); }
};

// Scalar path: one element at a time, identical arithmetic.  Used for the
// ragged tail of a tensor and for unaligned pointers.
template <class OP, class EPI, class WS>
__device__ __forceinline__ void reduce_scalar(const Seg<OP>& s, const EPI& epi, const WS& w, int K, int64_t e) {
  constexpr int SU = 16;  // clients in flight per lane: tiny tensors are latency-bound
  typename OP::acc_t acc = OP::first(as_global(s.src[0])[e], w[0]);
  int c = 1;
  for (; c + SU <= K; c += SU) {
    typename OP::in_t x[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) x[u] = as_global(s.src[c + u])[e];
#pragma unroll
    for (int u = 0; u < SU; ++u) acc = OP::step(acc, x[u], w[c + u]);
  }
  if (c < K) {  // remaining < SU clients: issue every load before the first add
    typename OP::in_t x[SU - 1];
#pragma unroll
    for (int u = 0; u < SU - 1; ++u)
      if (c + u < K) x[u] = as_global(s.src[c + u])[e];
#pragma unroll
    for (int u = 0; u < SU - 1; ++u)
      if (c + u < K) acc = OP::step(acc, x[u], w[c + u]);
  }
  epi.one(e, acc);
}

// Bounds-checked elements e, e + BS, ... (< e1), M at most, all chains in
// lockstep with SU clients' loads in flight; identical arithmetic to
// reduce_scalar, element by element.
template <class OP, int M, int BS, class EPI, class WS>
__device__ __forceinline__ void reduce_edge(const Seg<OP>& s, const EPI& epi, const WS& w, int K, int64_t e, int64_t e1) {
  constexpr int SU = (64 / M) < 1 ? 1 : ((64 / M) > 16 ? 16 : (64 / M));
  using in_t = typename OP::in_t;
  if (e >= e1) return;  // a lane past the end of a short last block owns nothing (and must load nothing)
  bool ok[M];
  typename OP::acc_t acc[M];
  {
    const auto p0 = as_global(s.src[0]);
    const auto w0 = w[0];
#pragma unroll
    for (int j = 0; j < M; ++j) {
      ok[j] = e + int64_t(j) * BS < e1;
      acc[j] = OP::first(p0[ok[j] ? e + int64_t(j) * BS : e], w0);
    }
  }
  // Out-of-range elements load a valid in-range address instead (e itself,
  // in range after the check above), so the loads need no predicate and
  // batch; their chains are discarded.
  int64_t idx[M];
#pragma unroll
  for (int j = 0; j < M; ++j) idx[j] = ok[j] ? e + int64_t(j) * BS : e;
  int c = 1;
  for (; c + SU <= K; c += SU) {
    in_t x[SU][M];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const auto p = as_global(s.src[c + u]);
#pragma unroll
      for (int j = 0; j < M; ++j) x[u][j] = p[idx[j]];
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const auto wu = w[c + u];
#pragma unroll
      for (int j = 0; j < M; ++j) acc[j] = OP::step(acc[j], x[u][j], wu);
    }
  }
  for (; c < K; ++c) {  // fewer than SU clients left
    const auto p = as_global(s.src[c]);
    const auto wc = w[c];
    in_t x[M];
#pragma unroll
    for (int j = 0; j < M; ++j) x[j] = p[idx[j]];
#pragma unroll
    for (int j = 0; j < M; ++j) acc[j] = OP::step(acc[j], x[j], wc);
  }
#pragma unroll
  for (int j = 0; j < M; ++j)
    if (ok[j]) epi.one(e + int64_t(j) * BS, acc[j]);
}

// One client's pack into a lane's E chains: through OP::step2 two elements at
// a time where the op has it (the packed-math form of the same arithmetic).
template <class OP, class = void>
struct HasStep2 : std::false_type {};
template <class OP>
struct HasStep2<OP, std::void_t<decltype(&OP::step2)>> : std::true_type {};

template <class OP, int E>
__device__ __forceinline__ void step_pack(typename OP::acc_t (&acc)[E], const Pack<typename OP::in_t, E>& x,
                                          typename OP::w_t w) {
  if constexpr (HasStep2<OP>::value && E % 2 == 0) {
#pragma unroll
    for (int e = 0; e < E; e += 2) OP::step2(acc[e], acc[e + 1], x.v[e], x.v[e + 1], w);
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = OP::step(acc[e], x.v[e], w);
  }
}

// Body of one workgroup of BS lanes: packs [pack0, pack0 + BS*V) of segment s.
template <class OP, int U, int V, bool NT, bool ALIGNED, int BS, class EPI, class WS>
__device__ __forceinline__ void reduce_block(const Seg<OP>& s, const EPI& epi, const WS& w, int K, int64_t pack0) {
  using in_t = typename OP::in_t;
  using w_t = typename OP::w_t;
  constexpr int E = 16 / sizeof(in_t);
  const int t = threadIdx.x;
  const int64_t full_packs = s.numel / E;

  if (ALIGNED && pack0 + int64_t(BS) * V <= full_packs) {
    // ---- fast path: every lane owns V whole 16-byte packs --------------------
    int64_t off[V];
#pragma unroll
    for (int v = 0; v < V; ++v) off[v] = (pack0 + v * BS + t) * E;

    typename EPI::Pre pre[V];
#pragma unroll
    for (int v = 0; v < V; ++v) pre[v] = epi.pre(off[v]);

    typename OP::acc_t acc[V][E];
    {
      const in_t* p = s.src[0];
      const w_t w0 = w[0];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        auto x = load_pack<in_t, NT>(p + off[v]);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[v][e] = OP::first(x.v[e], w0);
      }
    }
    int c = 1;
    for (; c + U <= K; c += U) {
      Pack<in_t, E> x[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const in_t* p = s.src[c + u];
#pragma unroll
        for (int v = 0; v < V; ++v) x[u][v] = load_pack<in_t, NT>(p + off[v]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const w_t wu = w[c + u];
#pragma unroll
        for (int v = 0; v < V; ++v) step_pack<OP, E>(acc[v], x[u][v], wu);
      }
    }
    if constexpr (U > 1) {
      if (c < K) {  // remaining < U clients (wave-uniform): all loads first, then the adds
        Pack<in_t, E> x[U - 1][V];
#pragma unroll
        for (int u = 0; u < U - 1; ++u)
          if (c + u < K) {
            const in_t* p = s.src[c + u];
#pragma unroll
            for (int v = 0; v < V; ++v) x[u][v] = load_pack<in_t, NT>(p + off[v]);
          }
#pragma unroll
        for (int u = 0; u < U - 1; ++u)
          if (c + u < K) {
            const w_t wu = w[c + u];
#pragma unroll
            for (int v = 0; v < V; ++v) step_pack<OP, E>(acc[v], x[u][v], wu);
          }
      }
    }
#pragma unroll
    for (int v = 0; v < V; ++v) epi.pack(off[v], acc[v], pre[v]);
  } else {
    // ---- edge path: element-wise with bounds ---------------------------------
    // The lane's V*E elements (e0 + t + j*BS) advance TOGETHER through the
    // client chain, so a ragged last block costs one chain, not V*E chains
    // one after another (that tail dominated small tensors with many clients).
    const int64_t e0 = pack0 * E;
    const int64_t e1 = min(s.numel, (pack0 + int64_t(BS) * V) * E);
    reduce_edge<OP, V * E, BS>(s, epi, w, K, e0 + t, e1);
  }
}

template <class OP, int U, int V, bool NT, bool ALIGNED, int BS, class EPI = StoreEpi<OP>,
          class WS = PtrW<typename OP::w_t>>
__global__ __launch_bounds__(BS) void reduce_kernel(Seg<OP> s, EPI epi, WS w, int K) {
  reduce_block<OP, U, V, NT, ALIGNED, BS>(s, epi, w, K, int64_t(blockIdx.x) * BS * V);
}

// Reduction fused with the server Adam / SGD epilogues (AdamEpi, SgdEpi):
// the prefetched optimizer operands sit in VGPRs across the client loop; cap
// the kernel at 128 VGPRs so 4 waves per SIMD stay resident (uncapped, Adam
// lands at 130 and SGD at 142-166 VGPRs, 3 waves).  Capped, the SGD kernel
// spills 6-16 VGPRs of its element-wise edge path to scratch, and still runs
// config 5 in 0.166 against 0.182 ms (tools/ab_libs.py, back to back,
// profiles/r05/ab/ab_cap.txt).
template <class OP, int U, int V, bool NT, bool ALIGNED, int BS, class EPI, class WS>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(4))) void reduce_fused_kernel(
    Seg<OP> s, EPI epi, WS w, int K) {
  reduce_block<OP, U, V, NT, ALIGNED, BS>(s, epi, w, K, int64_t(blockIdx.x) * BS * V);
}

#ifdef FEDAGG_TUNING
// XCD-contiguous tile order (tuning variant): workgroups are dispatched to the
// 8 XCDs round-robin, so block b runs on XCD b % 8; this remap gives each XCD
// one contiguous range of tiles instead of every eighth tile (a bijection for
// any grid size: XCD x takes q + (x < r) tiles, G = 8q + r).
template <class OP, int U, int V, bool NT, bool ALIGNED, int BS, class EPI, class WS>
__global__ __launch_bounds__(BS) void reduce_xcd_kernel(Seg<OP> s, EPI epi, WS w, int K) {
  const int64_t G = gridDim.x, b = blockIdx.x, q = G / 8, r = G % 8, x = b % 8;
  const int64_t tile = x * q + (x < r ? x : r) + b / 8;
  reduce_block<OP, U, V, NT, ALIGNED, BS>(s, epi, w, K, tile * BS * V);
}

// Grid-stride form: a resident grid walks the tiles, so no partial last wave of
// workgroups is left running alone at the end.
template <class OP, int U, int V, bool NT, int BS>
__global__ __launch_bounds__(BS) void reduce_persistent_kernel(Seg<OP> s, StoreEpi<OP> epi,
                                                               PtrW<typename OP::w_t> w, int K, int64_t tiles) {
  for (int64_t b = blockIdx.x; b < tiles; b += gridDim.x)
    reduce_block<OP, U, V, NT, true, BS>(s, epi, w, K, b * BS * V);
}

#endif  // FEDAGG_TUNING

// Multi-tensor form: blockIdx -> (segment, block within segment) by binary
// search over the prefix of per-segment block counts (wave-uniform, s_load).
template <class OP, int U, int V, bool NT, int BS>
__global__ __launch_bounds__(BS) void reduce_multi_kernel(
    const typename OP::in_t* const* __restrict__ src_tab, typename OP::out_t* const* __restrict__ out_tab,
    const int64_t* __restrict__ numel, const int64_t* __restrict__ block_begin, int T,
    const typename OP::w_t* __restrict__ wp, int K) {
  const PtrW<typename OP::w_t> w{wp};
  const int64_t b = blockIdx.x;
  int lo = 0, hi = T - 1;
  while (lo < hi) {  // largest s with block_begin[s] <= b
    const int mid = (lo + hi + 1) >> 1;
    if (block_begin[mid] <= b) lo = mid; else hi = mid - 1;
  }
  Seg<OP> s{src_tab + int64_t(lo) * K, numel[lo]};
  StoreEpi<OP> epi{out_tab[lo]};
  reduce_block<OP, U, V, NT, true, BS>(s, epi, w, K, (b - block_begin[lo]) * BS * V);
}

// Many clients over a small tensor (cross-device FedAvg: 1,000 clients x a
// 62K-element CNN): the element axis is all the parallelism there is (each
// element's client chain is sequential for bit-exactness), so a lane owns EL
// elements (a 2-, 4- or 8-byte pack, not 16) — up to 8x the lanes of the
// 16-byte tiles for 16-bit rows — and keeps U clients' loads in flight.  The
// wave then walks its chain in K/U memory round trips.
template <int B>
struct RawOf;
template <> struct RawOf<2> { using T = uint16_t; };
template <> struct RawOf<4> { using T = uint32_t; };
template <> struct RawOf<8> { using T = u32x2; };
template <> struct RawOf<16> { using T = u32x4; };

template <class OP, int U, int EL, bool ALIGNED, int BS, class WS>
__global__ __launch_bounds__(BS) void reduce_narrow_kernel(Seg<OP> s, StoreEpi<OP> epi, WS w, int K) {
  using in_t = typename OP::in_t;
  using raw_t = typename RawOf<EL * sizeof(in_t)>::T;
  const int64_t e0 = (int64_t(blockIdx.x) * BS + threadIdx.x) * EL;
  if (e0 >= s.numel) return;
  if (!ALIGNED || e0 + EL > s.numel) {
    reduce_edge<OP, EL, 1>(s, epi, w, K, e0, s.numel < e0 + EL ? s.numel : e0 + EL);
    return;
  }
  auto ld = [&](int c) {
    const raw_t r = __builtin_nontemporal_load(reinterpret_cast<const raw_t __attribute__((address_space(1)))*>(
        as_global(s.src[c]) + e0));
    Pack<in_t, EL> x;
    __builtin_memcpy(&x, &r, sizeof(r));
    return x;
  };
  typename OP::acc_t acc[EL];
  {
    const auto x = ld(0);
    const auto w0 = w[0];
#pragma unroll
    for (int j = 0; j < EL; ++j) acc[j] = OP::first(x.v[j], w0);
  }
  int c = 1;
  for (; c + U <= K; c += U) {
    Pack<in_t, EL> x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = ld(c + u);
#pragma unroll
    for (int u = 0; u < U; ++u) step_pack<OP, EL>(acc, x[u], w[c + u]);
  }
  if (c < K) {  // fewer than U clients left (wave-uniform): every load before the first add
    Pack<in_t, EL> x[U - 1];
#pragma unroll
    for (int u = 0; u < U - 1; ++u)
      if (c + u < K) x[u] = ld(c + u);
#pragma unroll
    for (int u = 0; u < U - 1; ++u)
      if (c + u < K) step_pack<OP, EL>(acc, x[u], w[c + u]);
  }
#pragma unroll
  for (int j = 0; j < EL; ++j) epi.one(e0 + j, acc[j]);
}

template <class OP, int U, int EL, int BS = 64, class WS = PtrW<typename OP::w_t>>
int launch_narrow(const typename OP::in_t* const* src, const WS& w, int32_t K, int64_t N, typename OP::out_t* out,
                  bool aligned, hipStream_t stream, const char* name) {
  const int64_t grid = ((N + EL - 1) / EL + BS - 1) / BS;
  if (grid > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, std::string(name) + ": N too large");
  Seg<OP> s{src, N};
  StoreEpi<OP> epi{out};
  if (aligned)
    hipLaunchKernelGGL((reduce_narrow_kernel<OP, U, EL, true, BS, WS>), dim3(unsigned(grid)), dim3(BS), 0, stream, s,
                       epi, w, K);
  else
    hipLaunchKernelGGL((reduce_narrow_kernel<OP, U, EL, false, BS, WS>), dim3(unsigned(grid)), dim3(BS), 0, stream, s,
                       epi, w, K);
  return check_launch(name);
}

// ---------------------------------------------------------------------------
// Shipped kernel configuration per op (chosen by tools/tune_wsum.py on MI355X).

// fp32 at 128 x 25.6M on MI355X: U4V4nt 6.44 TB/s vs U8V1nt 6.25 (profiles/r01_tune_variants_s2.json).
template <class OP> struct Cfg { static constexpr int U = 4, V = 4, BS = 256; static constexpr bool NT = true; };
// bf16 reference chain (round 5, after its packed rounding): one client per
// step per lane.  tools/tune_tiny.py, interleaved, bit-identical
// (profiles/r05/j/): 512 x 86.6M (config 4) 13.65 vs 14.04 ms for U4V4,
// 128 x 86.6M 3.20 vs 3.31, 64 x 86.6M 1.60 vs 1.66.
template <> struct Cfg<OpBF16Ref> { static constexpr int U = 1, V = 4, BS = 256; static constexpr bool NT = true; };
// ... and from 256 clients, eight packs per lane (U1V8: 272 VGPRs, one wave
// per SIMD, so ONE 256-lane workgroup per CU) when its workgroups fill their
// resident rounds: a U1V8 workgroup streams 16,384 elements of every client
// (16.8 MB at 512 clients, ~0.6 ms), so a last round that keeps only part of
// the CUs busy costs a large slice of the launch.  tools/ab_backtoback.py, 10
// launches back to back per sample (profiles/r05/m/, r05/q/), U1V8 vs U1V4 at
// 512 clients by rounds = workgroups / CUs: 86.6M (20.64 rounds) 13.32 vs
// 13.74 ms, 33.6M (8.0) 4.92 vs 4.99, 25.2M (6.0) 3.73 vs 3.77, 16.8M (4.0)
// 2.44 vs 2.50; but 60M (14.3) 9.50 vs 9.25, 43.3M (10.3) 6.94 vs 6.67, 21.6M
// (5.16) 3.82 vs 3.40, 10.8M (2.58) 1.93 vs 1.76.  So U1V8 where rounds /
// ceil(rounds) >= 0.97.  At 128 and 192 clients the two tie.  16-bit rows of
// 8M elements and more only (below, the narrow packs run).
constexpr int32_t kBF16WideFromClients = 256;
// The bf16 -> fp32 partial of the client-axis split (OpBF16F32Out, no
// roundings in the chain): U1V8 leads by more and tolerates a thinner last
// round.  U1V8 vs U1V4 vs U4V4: 128 x 86.6M (20.64 rounds) 3.37 / 3.62 / 3.68
// ms, 64 x 86.6M 1.75 / 1.93 / 1.97, 256 x 86.6M 6.71 / 6.94 / 7.00, 128 x
// 43.3M (10.3) 1.70 / 1.78 / 1.82; 128 x 21.6M (5.16) 0.90 / 0.875 / 0.872.
// So U1V8 from 32 clients where rounds / ceil(rounds) >= 0.9.
constexpr int32_t kF32OutWideFromClients = 32;
// The fp32-accumulated bf16 chain (acc_mode fp32, OpBF16Acc32) sits between
// the two (profiles/r05/t/): U1V8 / U1V4 / U4V4 at 512 x 86.6M 13.12 / 13.60
// / 14.00 ms, 64 x 86.6M 1.69 / 1.77 / 1.82, 128 x 86.6M 3.42 / 3.43 / 3.45,
// 512 x 43.3M (10.3 rounds) 6.56 / 6.46 / 6.62, 512 x 21.6M 3.54 / 3.30 /
// (mid tiles) 3.30.  U1V4 tiles, U1V8 from 32 clients at a fill >= 0.97.
template <> struct Cfg<OpBF16Acc32> { static constexpr int U = 1, V = 4, BS = 256; static constexpr bool NT = true; };

// CUs of the current device (cached per device ordinal).
int device_cus() {
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
// Fill of the last resident round when every CU holds one workgroup of
// `elems_per_wg` elements: rounds / ceil(rounds).
double round_fill(int64_t N, int64_t elems_per_wg) {
  const double rounds = double((N + elems_per_wg - 1) / elems_per_wg) / device_cus();
  return rounds / std::ceil(rounds);
}

// Tensors too small to fill the chip with 4,096-element tiles (configs 1-2,
// LoRA-sized keys) use 256-element tiles of 64 lanes with 16 clients in flight
// per lane: ~16x more workgroups and one memory round trip per 16 clients.
struct SmallCfg { static constexpr int U = 16, V = 1, BS = 64; static constexpr bool NT = true; };
// shipped-tile workgroups below which SmallCfg is used.  Round 3 re-measured
// the sizes between configs 2 and 5 (the per-rank shards of strong scaling,
// tools/tune_mid.py, profiles/r03/tune_mid.txt, 25 interleaved rounds): the
// small tiles lead up to 128 blocks and trail U2V4 by 8-10 % at 256 blocks
// and U1V4 by 5-7 % at 512-1,023 blocks, where round 2 still used them.
constexpr int64_t kSmallBelowBlocks = 256;
// 256-511 blocks: two clients in flight per lane (U2V4), 0-1 % off the best
// variant at K = 32, 64 and 128; U1V4 trails it there by 10-17 %.
struct Mid2Cfg { static constexpr int U = 2, V = 4, BS = 256; static constexpr bool NT = true; };
constexpr int64_t kMid2BelowBlocks = 512;

// Many clients over a tensor too small to give every CU a workgroup (e.g. 1,000
// clients x a 7,850-element model): each lane's chain over the clients is a
// sequence of memory round trips, so twice the clients in flight halves it.
// Since round 3 only the 8-byte element types (fp64, int64) take this tile:
// 16-bit and fp32 rows go to the narrow packs below (round 2's 16-bit Tiny
// tiles also sat at 262-266 VGPRs, one wave per SIMD).
struct TinyCfg { static constexpr int U = 32, V = 1, BS = 64; static constexpr bool NT = true; };
constexpr int64_t kTinyBelowElems = 65536;  // fewer than 256 small-tile workgroups
constexpr int32_t kTinyFromClients = 48;

// Mid-sized launches (1,024 to 4,096 tiles: every tile resident at once or
// nearly so) stream one client at a time per lane (56 VGPRs instead of 94).
// tools/tune_wsum.py and tools/adam_probe.py on MI355X: 64 x 4.19M (config 5)
// FedAvg 0.160 vs 0.171 ms, fused SGD 0.168 vs 0.177 ms, fused Adam 0.175 vs
// 0.197 ms; 128 x 4.19M 0.317 vs 0.348 ms; 128 x 16.8M 1.271 vs 1.298 ms.  At
// config 3 (6,253 tiles) U4V4 stays ahead (2.047 vs 2.067 ms).
struct MidCfg { static constexpr int U = 1, V = 4, BS = 256; static constexpr bool NT = true; };
constexpr int64_t kMidUpToBlocks = 4096;

template <class OP>
int64_t blocks_for(int64_t numel) {
  constexpr int E = 16 / sizeof(typename OP::in_t);
  const int64_t packs = (numel + E - 1) / E;
  const int64_t per = int64_t(Cfg<OP>::BS) * Cfg<OP>::V;
  return (packs + per - 1) / per;
}

template <class OP, int U, int V, bool NT, int BS = 256, class WS = PtrW<typename OP::w_t>>
int launch_uvn(const typename OP::in_t* const* src, const WS& w, int32_t K, int64_t N, typename OP::out_t* out,
               bool aligned, hipStream_t stream, const char* name) {
  constexpr int E = 16 / sizeof(typename OP::in_t);
  const int64_t packs = (N + E - 1) / E;
  const int64_t per = int64_t(BS) * V;
  const int64_t grid = (packs + per - 1) / per;
  if (grid > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, std::string(name) + ": N too large");
  Seg<OP> s{src, N};
  StoreEpi<OP> epi{out};
  if (aligned) {
    hipLaunchKernelGGL((reduce_kernel<OP, U, V, NT, true, BS, StoreEpi<OP>, WS>), dim3(unsigned(grid)), dim3(BS), 0,
                       stream, s, epi, w, K);
  } else {
    hipLaunchKernelGGL((reduce_kernel<OP, U, V, NT, false, BS, StoreEpi<OP>, WS>), dim3(unsigned(grid)), dim3(BS), 0,
                       stream, s, epi, w, K);
  }
  return check_launch(name);
}

// Narrow packs (reduce_narrow_kernel) where the 16-byte tiles leave too few
// lanes (tools/tune_tiny.py, profiles/r03/tiny/: every variant bit-identical).
//   - 16-bit rows below 8M elements, any K: a 16-byte pack is 8 elements, so
//     the wide tiles give a 1M-element tensor 2,048 64-lane blocks, each lane
//     walking 8 reference chains.  Four-byte packs (EL = 2) give 4x the
//     lanes: 1,000 x 62,006 bf16 0.132 -> 0.050 ms (EL = 1, 32 clients in
//     flight, from 512 clients), 128 x 1M 0.057 -> 0.044 ms, 32 x 4M 0.052 ->
//     0.047 ms; from 16M elements the wide tiles lead again.
//   - fp32 below 1M elements with at least 48 clients: 8-byte packs (4-byte
//     ones from 32K elements while the tensor is below the Tiny bound):
//     4,096 x 7,850 0.215 -> 0.138 ms, 1,000 x 200K 0.144 -> 0.125 ms.
constexpr int64_t kNarrow16BelowElems = int64_t(8) << 20;
constexpr int64_t kNarrow32BelowElems = int64_t(1) << 20;
template <class OP, class WS>
int launch_narrow_policy(const typename OP::in_t* const* s, const WS& w, int32_t K, int64_t N,
                         typename OP::out_t* o, bool al, hipStream_t st, const char* name) {
  if constexpr (sizeof(typename OP::in_t) == 2) {
    if (K >= 512 && N < kTinyBelowElems) return launch_narrow<OP, 32, 1, 64, WS>(s, w, K, N, o, al, st, name);
    if (K >= 512 && N < kNarrow32BelowElems) return launch_narrow<OP, 32, 2, 64, WS>(s, w, K, N, o, al, st, name);
    return launch_narrow<OP, 16, 2, 64, WS>(s, w, K, N, o, al, st, name);
  } else {
    if (N >= 32768 && N < kTinyBelowElems) return launch_narrow<OP, 32, 1, 64, WS>(s, w, K, N, o, al, st, name);
    return launch_narrow<OP, 32, 2, 64, WS>(s, w, K, N, o, al, st, name);
  }
}
template <class OP>
constexpr bool narrow_ok() {  // 4- and 8-byte packs of the element type
  return sizeof(typename OP::in_t) == 2 || sizeof(typename OP::in_t) == 4;
}

template <class OP, class WS>
int launch_ws(const typename OP::in_t* const* s, const WS& w, int32_t K, int64_t N, typename OP::out_t* o, bool al,
              hipStream_t st, const char* name) {
  const int64_t blocks = blocks_for<OP>(N);
  if constexpr (narrow_ok<OP>()) {
    if (sizeof(typename OP::in_t) == 2 ? N < kNarrow16BelowElems : (N < kNarrow32BelowElems && K >= kTinyFromClients))
      return launch_narrow_policy<OP, WS>(s, w, K, N, o, al, st, name);
  }
  if constexpr (!narrow_ok<OP>()) {  // 2- and 4-byte rows never reach it (narrow packs above)
    if (N < kTinyBelowElems && K >= kTinyFromClients)
      return launch_uvn<OP, TinyCfg::U, TinyCfg::V, TinyCfg::NT, TinyCfg::BS, WS>(s, w, K, N, o, al, st, name);
  }
  if constexpr (std::is_same_v<OP, OpBF16Ref> || std::is_same_v<OP, OpBF16F32Out> ||
                std::is_same_v<OP, OpBF16Acc32>) {
    constexpr bool ref = std::is_same_v<OP, OpBF16Ref>;
    constexpr double min_fill = std::is_same_v<OP, OpBF16F32Out> ? 0.9 : 0.97;
    if (K >= (ref ? kBF16WideFromClients : kF32OutWideFromClients) && blocks >= kMid2BelowBlocks &&
        round_fill(N, int64_t(256) * 8 * 8) >= min_fill)
      return launch_uvn<OP, 1, 8, true, 256, WS>(s, w, K, N, o, al, st, name);
  }
  if (blocks < kSmallBelowBlocks)
    return launch_uvn<OP, SmallCfg::U, SmallCfg::V, SmallCfg::NT, SmallCfg::BS, WS>(s, w, K, N, o, al, st, name);
  if (blocks < kMid2BelowBlocks)
    return launch_uvn<OP, Mid2Cfg::U, Mid2Cfg::V, Mid2Cfg::NT, Mid2Cfg::BS, WS>(s, w, K, N, o, al, st, name);
  if (blocks <= kMidUpToBlocks)
    return launch_uvn<OP, MidCfg::U, MidCfg::V, MidCfg::NT, MidCfg::BS, WS>(s, w, K, N, o, al, st, name);
  return launch_uvn<OP, Cfg<OP>::U, Cfg<OP>::V, Cfg<OP>::NT, Cfg<OP>::BS, WS>(s, w, K, N, o, al, st, name);
}

// Any epilogue / weight source, shipped or small-tensor tiles by size.
template <class OP, class EPI, class WS, int U, int V, bool NT, int BS>
int launch_epi_cfg(const Seg<OP>& s, const EPI& epi, const WS& w, int32_t K, bool aligned, hipStream_t st,
                   const char* name) {
  constexpr int E = 16 / sizeof(typename OP::in_t);
  const int64_t grid = ((s.numel + E - 1) / E + int64_t(BS) * V - 1) / (int64_t(BS) * V);
  if (grid > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, std::string(name) + ": N too large");
  if (aligned) {
    hipLaunchKernelGGL((reduce_kernel<OP, U, V, NT, true, BS, EPI, WS>), dim3(unsigned(grid)), dim3(BS), 0, st, s, epi,
                       w, K);
  } else {
    hipLaunchKernelGGL((reduce_kernel<OP, U, V, NT, false, BS, EPI, WS>), dim3(unsigned(grid)), dim3(BS), 0, st, s,
                       epi, w, K);
  }
  return check_launch(name);
}

template <class OP, class EPI, class WS>
int launch_epi(const Seg<OP>& s, const EPI& epi, const WS& w, int32_t K, bool aligned, hipStream_t st,
               const char* name) {
  const int64_t blocks = blocks_for<OP>(s.numel);
  if (blocks < kSmallBelowBlocks)
    return launch_epi_cfg<OP, EPI, WS, SmallCfg::U, SmallCfg::V, SmallCfg::NT, SmallCfg::BS>(s, epi, w, K, aligned,
                                                                                            st, name);
  if (blocks < kMid2BelowBlocks)
    return launch_epi_cfg<OP, EPI, WS, Mid2Cfg::U, Mid2Cfg::V, Mid2Cfg::NT, Mid2Cfg::BS>(s, epi, w, K, aligned, st,
                                                                                        name);
  if (blocks <= kMidUpToBlocks)
    return launch_epi_cfg<OP, EPI, WS, MidCfg::U, MidCfg::V, MidCfg::NT, MidCfg::BS>(s, epi, w, K, aligned, st, name);
  return launch_epi_cfg<OP, EPI, WS, Cfg<OP>::U, Cfg<OP>::V, Cfg<OP>::NT, Cfg<OP>::BS>(s, epi, w, K, aligned, st,
                                                                                      name);
}

// Weights passed in the kernel arguments (flags & FEDAGG_HOST_WEIGHTS): w is a
// HOST array of K <= kInlineK values, copied into the launch packet.
template <class T>
bool inline_weights(const void* w, int32_t K, InlW<T>* out) {
  if (K > kInlineK) return false;
  memcpy(out->v, w, size_t(K) * sizeof(T));
  return true;
}

template <class OP>
int launch(const void* const* src, const void* w, int32_t K, int64_t N, void* out, uint32_t flags,
           fedagg_stream_t stream, const char* name, bool need_w = true) {
  if (K < 1 || N < 0) return set_error(FEDAGG_EINVAL, std::string(name) + ": K must be >= 1 and N >= 0");
  if (!src || !out || (need_w && !w)) return set_error(FEDAGG_EINVAL, std::string(name) + ": null pointer");
  if (N == 0) return FEDAGG_OK;
  auto s = reinterpret_cast<const typename OP::in_t* const*>(src);
  auto o = reinterpret_cast<typename OP::out_t*>(out);
  const bool al = (flags & FEDAGG_ALIGNED16) != 0;
  auto st = reinterpret_cast<hipStream_t>(stream);
  using w_t = typename OP::w_t;
  if (w && (flags & FEDAGG_HOST_WEIGHTS)) {
    InlW<w_t> iw;
    if (!inline_weights<w_t>(w, K, &iw))
      return set_error(FEDAGG_EINVAL, std::string(name) + ": FEDAGG_HOST_WEIGHTS needs K <= 256");
    return launch_ws<OP>(s, iw, K, N, o, al, st, name);
  }
  return launch_ws<OP>(s, PtrW<w_t>{reinterpret_cast<const w_t*>(w)}, K, N, o, al, st, name);
}

// ---------------------------------------------------------------------------
// Tuning build only (tools/build_tuning.py compiles this file with
// -DFEDAGG_TUNING into tools/_build/libfedagg_tuning.so): the A/B tables the
// shipped tile shapes were chosen from.  The product library carries none of it.
#ifdef FEDAGG_TUNING
#define FEDAGG_TUNE_BF16_F32OUT 0x101  // bf16 rows, fp32 partial out
#define FEDAGG_TUNE_BF16_ACC32 0x102   // bf16 rows, fp32 accumulation

// ---------------------------------------------------------------------------
// Tuning table for the fp32 kernel (fedagg_wsum_f32_variant).

struct Variant {
  const char* name;
  int (*fn)(const float* const*, const float*, int32_t, int64_t, float*, hipStream_t);
};

template <int U, int V, bool NT, int BS>
int variant_fn(const float* const* src, const float* w, int32_t K, int64_t N, float* out, hipStream_t st) {
  return launch_uvn<OpF32, U, V, NT, BS>(src, PtrW<float>{w}, K, N, out, true, st, "fedagg_wsum_f32_variant");
}

template <int U, int V, int BS>
int xcd_fn(const float* const* src, const float* w, int32_t K, int64_t N, float* out, hipStream_t st) {
  const int64_t grid = ((N + 3) / 4 + int64_t(BS) * V - 1) / (int64_t(BS) * V);
  Seg<OpF32> s{src, N};
  hipLaunchKernelGGL((reduce_xcd_kernel<OpF32, U, V, true, true, BS, StoreEpi<OpF32>, PtrW<float>>), dim3(unsigned(grid)),
                     dim3(BS), 0, st, s, StoreEpi<OpF32>{out}, PtrW<float>{w}, K);
  return check_launch("xcd");
}

template <int U, int V, int BS, int PER_CU>
int persistent_fn(const float* const* src, const float* w, int32_t K, int64_t N, float* out, hipStream_t st) {
  constexpr int E = 4;
  const int64_t tiles = ((N + E - 1) / E + int64_t(BS) * V - 1) / (int64_t(BS) * V);
  const int64_t grid = tiles < 256 * PER_CU ? tiles : 256 * PER_CU;
  Seg<OpF32> s{src, N};
  StoreEpi<OpF32> epi{out};
  hipLaunchKernelGGL((reduce_persistent_kernel<OpF32, U, V, true, BS>), dim3(unsigned(grid)), dim3(BS), 0, st, s, epi,
                     PtrW<float>{w}, K, tiles);
  return check_launch("persistent");
}

// what fedagg_wsum_f32 dispatches for this size (Tiny / Small / Mid / shipped tiles)
int shipped_fn(const float* const* src, const float* w, int32_t K, int64_t N, float* out, hipStream_t st) {
  return launch_ws<OpF32>(src, PtrW<float>{w}, K, N, out, true, st, "fedagg_wsum_f32_variant");
}

const Variant kVariants[] = {
    {"U8V1nt", variant_fn<8, 1, true, 256>},      {"U8V2nt", variant_fn<8, 2, true, 256>},
    {"U4V4nt", variant_fn<4, 4, true, 256>},      {"U2V4nt", variant_fn<2, 4, true, 256>},
    {"U8V4nt", variant_fn<8, 4, true, 256>},      {"U2V8nt", variant_fn<2, 8, true, 256>},
    {"U4V8nt", variant_fn<4, 8, true, 256>},      {"U1V8nt", variant_fn<1, 8, true, 256>},
    {"U4V4nt_b128", variant_fn<4, 4, true, 128>}, {"U4V4nt_b512", variant_fn<4, 4, true, 512>},
    {"U2V4nt_b512", variant_fn<2, 4, true, 512>}, {"U4V2nt_b1024", variant_fn<4, 2, true, 1024>},
    {"U4V4", variant_fn<4, 4, false, 256>},
    {"U4V4nt_p4", persistent_fn<4, 4, 256, 4>},   {"U4V4nt_p5", persistent_fn<4, 4, 256, 5>},
    {"U4V4nt_p8", persistent_fn<4, 4, 256, 8>},   {"U4V2nt_p8", persistent_fn<4, 2, 256, 8>},
    {"U1V4nt", variant_fn<1, 4, true, 256>},      {"U1V2nt", variant_fn<1, 2, true, 256>},
    {"U2V2nt", variant_fn<2, 2, true, 256>},
    {"U4V4nt_xcd", xcd_fn<4, 4, 256>},            {"U1V4nt_xcd", xcd_fn<1, 4, 256>},
    {"U16V1nt_b64", variant_fn<16, 1, true, 64>}, {"U8V1nt_b64", variant_fn<8, 1, true, 64>},
    {"U8V2nt_b64", variant_fn<8, 2, true, 64>},   {"U4V4nt_b64", variant_fn<4, 4, true, 64>},
    {"U2V4nt_b128", variant_fn<2, 4, true, 128>}, {"U1V4nt_b128", variant_fn<1, 4, true, 128>},
    {"shipped", shipped_fn},
};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

// Tuning table for many clients over small tensors (fedagg_wsum_tiny_variant):
// fp32 and bf16 (reference chain), 16-byte tiles against narrow packs.
using TinyFn = int (*)(const void* const*, const float*, int32_t, int64_t, void*, hipStream_t);
struct TinyVariant {
  const char* name;
  TinyFn f32, bf16;
  TinyFn bf16f32 = nullptr;  // bf16 rows, fp32 partial out (client-axis pre-reduction); wide tiles only
  TinyFn bf16acc32 = nullptr;  // bf16 rows, fp32 accumulation, bf16 out (acc_mode fp32); wide tiles only
};
template <class OP, int U, int EL>
int tiny_narrow_fn(const void* const* src, const float* w, int32_t K, int64_t N, void* out, hipStream_t st) {
  constexpr int BS = 64;
  const int64_t grid = ((N + EL - 1) / EL + BS - 1) / BS;
  hipLaunchKernelGGL((reduce_narrow_kernel<OP, U, EL, true, BS, PtrW<float>>), dim3(unsigned(grid)), dim3(BS), 0, st,
                     Seg<OP>{reinterpret_cast<const typename OP::in_t* const*>(src), N},
                     StoreEpi<OP>{reinterpret_cast<typename OP::out_t*>(out)}, PtrW<float>{w}, K);
  return check_launch("fedagg_wsum_tiny_variant");
}
template <class OP, int U>
int tiny_wide_fn(const void* const* src, const float* w, int32_t K, int64_t N, void* out, hipStream_t st) {
  return launch_uvn<OP, U, 1, true, 64>(reinterpret_cast<const typename OP::in_t* const*>(src), PtrW<float>{w}, K, N,
                                        reinterpret_cast<typename OP::out_t*>(out), true, st,
                                        "fedagg_wsum_tiny_variant");
}
template <class OP, int U, int V, int BS>
int tiny_uv_fn(const void* const* src, const float* w, int32_t K, int64_t N, void* out, hipStream_t st) {
  return launch_uvn<OP, U, V, true, BS>(reinterpret_cast<const typename OP::in_t* const*>(src), PtrW<float>{w}, K, N,
                                        reinterpret_cast<typename OP::out_t*>(out), true, st,
                                        "fedagg_wsum_tiny_variant");
}
// Round 5 A/B of the bf16 reference chain's instruction form: the rounding
// into the LOW half of v_cvt_pk_bf16_f32 plus a shift / mask back to fp32, one
// element at a time (what shipped until round 5), against the shipped
// high-half rounding with OpBF16Ref::step2's packed mul / add.  Bit-identical.
struct OpBF16RefLowHalf {
  using in_t = uint16_t; using out_t = uint16_t; using acc_t = float; using w_t = float;
  static __device__ __forceinline__ float r(float f) {
    const __bf16 b = static_cast<__bf16>(f);
    return bf16_to_f32(__builtin_bit_cast(uint16_t, b));
  }
  static __device__ __forceinline__ acc_t first(in_t x, w_t w) { return r(bf16_to_f32(x) * w); }
  static __device__ __forceinline__ acc_t step(acc_t a, in_t x, w_t w) { return r(a + r(bf16_to_f32(x) * w)); }
  static __device__ __forceinline__ out_t fin(acc_t a) { return f32_to_bf16(a); }
};
template <class OP>
int tiny_shipped_fn(const void* const* src, const float* w, int32_t K, int64_t N, void* out, hipStream_t st) {
  return launch_ws<OP>(reinterpret_cast<const typename OP::in_t* const*>(src), PtrW<float>{w}, K, N,
                       reinterpret_cast<typename OP::out_t*>(out), true, st, "fedagg_wsum_tiny_variant");
}
#define FEDAGG_TINY_NARROW(U, EL) \
  { "EL" #EL "_U" #U, tiny_narrow_fn<OpF32, U, EL>, tiny_narrow_fn<OpBF16Ref, U, EL> }
// (round 4: the entries that needed 258-266 VGPRs, wide_U32 and EL4_U64, one
// wave per SIMD and slower everywhere in profiles/r03/tiny/, are no longer
// instantiated)
const TinyVariant kTinyVariants[] = {
    {"shipped", tiny_shipped_fn<OpF32>, tiny_shipped_fn<OpBF16Ref>, tiny_shipped_fn<OpBF16F32Out>, tiny_shipped_fn<OpBF16Acc32>},
    {"wide_U16", tiny_wide_fn<OpF32, 16>, tiny_wide_fn<OpBF16Ref, 16>, tiny_wide_fn<OpBF16F32Out, 16>, tiny_wide_fn<OpBF16Acc32, 16>},
    {"U4V4", tiny_uv_fn<OpF32, 4, 4, 256>, tiny_uv_fn<OpBF16Ref, 4, 4, 256>, tiny_uv_fn<OpBF16F32Out, 4, 4, 256>, tiny_uv_fn<OpBF16Acc32, 4, 4, 256>},
    {"U4V4_lowhalf", tiny_uv_fn<OpF32, 4, 4, 256>, tiny_uv_fn<OpBF16RefLowHalf, 4, 4, 256>},
    {"U1V4", tiny_uv_fn<OpF32, 1, 4, 256>, tiny_uv_fn<OpBF16Ref, 1, 4, 256>, tiny_uv_fn<OpBF16F32Out, 1, 4, 256>, tiny_uv_fn<OpBF16Acc32, 1, 4, 256>},
    {"U1V4_lowhalf", tiny_uv_fn<OpF32, 1, 4, 256>, tiny_uv_fn<OpBF16RefLowHalf, 1, 4, 256>},
    {"U2V4", tiny_uv_fn<OpF32, 2, 4, 256>, tiny_uv_fn<OpBF16Ref, 2, 4, 256>, tiny_uv_fn<OpBF16F32Out, 2, 4, 256>, tiny_uv_fn<OpBF16Acc32, 2, 4, 256>},
    {"U1V8", tiny_uv_fn<OpF32, 1, 8, 256>, tiny_uv_fn<OpBF16Ref, 1, 8, 256>, tiny_uv_fn<OpBF16F32Out, 1, 8, 256>, tiny_uv_fn<OpBF16Acc32, 1, 8, 256>},
    {"U1V2", tiny_uv_fn<OpF32, 1, 2, 256>, tiny_uv_fn<OpBF16Ref, 1, 2, 256>, tiny_uv_fn<OpBF16F32Out, 1, 2, 256>, tiny_uv_fn<OpBF16Acc32, 1, 2, 256>},
    {"U2V2", tiny_uv_fn<OpF32, 2, 2, 256>, tiny_uv_fn<OpBF16Ref, 2, 2, 256>, tiny_uv_fn<OpBF16F32Out, 2, 2, 256>, tiny_uv_fn<OpBF16Acc32, 2, 2, 256>},
    {"U8V1", tiny_uv_fn<OpF32, 8, 1, 256>, tiny_uv_fn<OpBF16Ref, 8, 1, 256>, tiny_uv_fn<OpBF16F32Out, 8, 1, 256>, tiny_uv_fn<OpBF16Acc32, 8, 1, 256>},
    {"U4V2", tiny_uv_fn<OpF32, 4, 2, 256>, tiny_uv_fn<OpBF16Ref, 4, 2, 256>, tiny_uv_fn<OpBF16F32Out, 4, 2, 256>, tiny_uv_fn<OpBF16Acc32, 4, 2, 256>},
    FEDAGG_TINY_NARROW(16, 1), FEDAGG_TINY_NARROW(32, 1), FEDAGG_TINY_NARROW(64, 1),
    FEDAGG_TINY_NARROW(16, 2), FEDAGG_TINY_NARROW(32, 2), FEDAGG_TINY_NARROW(64, 2),
    FEDAGG_TINY_NARROW(16, 4), FEDAGG_TINY_NARROW(32, 4),
};
#undef FEDAGG_TINY_NARROW
constexpr int kNumTinyVariants = sizeof(kTinyVariants) / sizeof(kTinyVariants[0]);
#endif  // FEDAGG_TUNING

// ---------------------------------------------------------------------------
// fp32 -> bf16 / f16 rounding of a reduced shard (the client-axis multi-GPU
// mode accumulates bf16 clients in fp32 and rounds once, after the exchange).

template <bool BF16>
__global__ __launch_bounds__(kBlock) void round_f32_kernel(const float* __restrict__ in, uint16_t* __restrict__ out,
                                                           int64_t n) {
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride)
    out[i] = BF16 ? f32_to_bf16(in[i]) : f32_to_f16(in[i]);
}

// ---------------------------------------------------------------------------
// FedOpt SGD(+momentum) epilogue.

__global__ __launch_bounds__(kBlock) void fedopt_sgd_kernel(float* __restrict__ p, float* __restrict__ mom,
                                                            const float* __restrict__ avg, int64_t n, float neg_lr,
                                                            float m, int first) {
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    const float po = p[i];
    const float g = po - avg[i];
    float b = g;
    if (mom) {
      if (!first) b = mom[i] * m + g;  // two roundings (-ffp-contract=off): mul_ then add_
      mom[i] = b;
    }
    p[i] = __builtin_fmaf(b, neg_lr, po);  // add_(buf, alpha=-lr): vectorised fmadd
  }
}

}  // namespace

namespace {
// Persistent workers for the host packs (fedagg_host_pack / _unpack).  Every
// arriving client is one pack per dtype group, and a round spread over G GPUs
// (fedml_amd.multidev) packs each device's keys from its own Python thread at
// the same time: spawning 8 threads per call cost ~0.1-0.2 ms each time, and
// one shared job slot would serialize the shards.  Callers queue a batch of
// parts, work on it themselves, and idle workers join in; a batch leaves the
// queue when its parts are all claimed, and its caller returns once every
// part has run and no worker still holds it.
//
// Fork: the workers do not exist in a child process and the pool's mutex may
// have been held by one of them at the fork, so a pthread_atfork child
// handler drops the pool (leaked, never touched again) and the child's first
// pack builds its own.
class PackPool {
 public:
  static PackPool& get() {
    for (;;) {
      PackPool* p = pool_.load(std::memory_order_acquire);
      if (p) return *p;
      int idle = 0;
      if (creating_.compare_exchange_strong(idle, 1)) {
        static const int registered = pthread_atfork(nullptr, nullptr, [] {
          pool_.store(nullptr);
          creating_.store(0);
        });
        (void)registered;
        p = new PackPool(15);  // + the caller: 16, the GPU box's CPU share
        pool_.store(p, std::memory_order_release);
        creating_.store(0);
        return *p;
      }
      std::this_thread::yield();
    }
  }
  void run(int parts, const std::function<void(int)>& fn) {
    if (parts <= 1) {
      if (parts == 1) fn(0);
      return;
    }
    Batch b;
    b.fn = &fn;
    b.parts = parts;
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(&b);
    }
    cv_.notify_all();
    for (int part = b.next.fetch_add(1); part < parts; part = b.next.fetch_add(1)) {
      fn(part);
      b.done.fetch_add(1);
    }
    std::unique_lock<std::mutex> lk(mu_);
    for (size_t i = 0; i < q_.size(); ++i)
      if (q_[i] == &b) {
        q_.erase(q_.begin() + std::ptrdiff_t(i));
        break;
      }
    b.cv.wait(lk, [&] { return b.done.load() == parts && b.active == 0; });
  }

 private:
  struct Batch {
    const std::function<void(int)>* fn = nullptr;
    int parts = 0;
    int active = 0;  // workers holding this batch (guarded by mu_)
    std::atomic<int> next{0}, done{0};
    std::condition_variable cv;
  };
  explicit PackPool(int n) {
    for (int i = 0; i < n; ++i) std::thread([this] { loop(); }).detach();
  }
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return !q_.empty(); });
      Batch* b = q_.front();
      if (b->next.load() >= b->parts) {  // every part claimed: nothing left to join
        q_.erase(q_.begin());
        continue;
      }
      ++b->active;
      lk.unlock();
      for (int part = b->next.fetch_add(1); part < b->parts; part = b->next.fetch_add(1)) {
        (*b->fn)(part);
        b->done.fetch_add(1);
      }
      lk.lock();
      if (--b->active == 0) b->cv.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Batch*> q_;
  static std::atomic<PackPool*> pool_;
  static std::atomic<int> creating_;
};
std::atomic<PackPool*> PackPool::pool_{nullptr};
std::atomic<int> PackPool::creating_{0};

// Host copy with non-temporal 16-byte stores for the bulk: the staging rows
// are read next by the GPU's DMA (and the unpacked host tensors by whoever
// sends them), never by this core, so the stores skip the cache instead of
// reading every destination line first.  glibc's memcpy switches to such
// stores only for copies of several MB; config 5's 131 KB keys packed at
// 45 GB/s with it (tools/profile_arrival.py).
void copy_nt(char* dst, const char* src, size_t n) {
  if (n < 4096) {
    memcpy(dst, src, n);
    return;
  }
  const size_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
  memcpy(dst, src, head);
  dst += head;
  src += head;
  n -= head;
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
  }
  memcpy(dst + i, src + i, n - i);
}

// Parallel copy of n byte ranges: range i goes from src_base[i] to dst_base[i]
// (nbytes[i] bytes).  The total is cut into `threads` contiguous slices, run
// on the persistent PackPool; each slice ends with a store fence, so its
// streamed stores are visible before the caller issues the DMA.
template <class SrcAt, class DstAt>
void parallel_ranges(int32_t n, const int64_t* nbytes, int32_t threads, SrcAt src_at, DstAt dst_at) {
  int64_t total = 0;
  for (int32_t i = 0; i < n; ++i) total += nbytes[i];
  if (total == 0) return;
  int32_t T = threads < 1 ? 1 : threads;
  if (total < (4ll << 20)) T = 1;  // below ~4 MiB one thread beats spawning
  auto work = [&](int64_t b0, int64_t b1) {
    int64_t pos = 0;
    for (int32_t i = 0; i < n && pos < b1; ++i) {
      const int64_t lo = pos, hi = pos + nbytes[i];
      pos = hi;
      if (hi <= b0) continue;
      const int64_t a = lo > b0 ? lo : b0, b = hi < b1 ? hi : b1;
      copy_nt(dst_at(i) + (a - lo), src_at(i) + (a - lo), size_t(b - a));
    }
    _mm_sfence();
  };
  if (T == 1) {
    work(0, total);
    return;
  }
  const int64_t per = ((total + T - 1) / T + 4095) & ~int64_t(4095);
  const int parts = int((total + per - 1) / per);
  auto part = [&](int t) {
    const int64_t b0 = int64_t(t) * per, b1 = b0 + per < total ? b0 + per : total;
    work(b0, b1);
  };
  const char* sp = getenv("FEDAGG_PACK_SPAWN");  // "1": round 3's thread per part and call (A/B, read per call)
  if (sp && sp[0] == '1') {
    std::vector<std::thread> pool;
    for (int t = 0; t < parts; ++t) pool.emplace_back(part, t);
    for (auto& th : pool) th.join();
    return;
  }
  PackPool::get().run(parts, part);
}

int check_ranges(int32_t n, const void* a, const void* b, const int64_t* offs, const int64_t* nbytes,
                 const char* what) {
  if (n < 0 || (n > 0 && (!a || !b || !offs || !nbytes))) return set_error(FEDAGG_EINVAL, std::string(what) + ": bad argument");
  for (int32_t i = 0; i < n; ++i)
    if (nbytes[i] < 0 || offs[i] < 0) return set_error(FEDAGG_EINVAL, std::string(what) + ": negative size");
  return FEDAGG_OK;
}
// (the anonymous namespace continues: the small-round machinery below is internal too)

// ---------------------------------------------------------------------------
// One small host-resident round, host to host (fedagg_host_round_f32).
//
// Config 1 (4 clients x 7,850 fp32) is 125 KB: a PCIe round trip plus the
// launch and completion latencies, not bytes, decide its time, and every
// torch-level step around them (pinned copies, events, stream bookkeeping)
// costs as much as the reduction.  So the whole round is one call: pack the
// clients into a coherent pinned image [K][L] (L = the model's keys, 16-byte
// aligned, padded to 64 elements), reduce, and unpack the result into the
// caller's host tensors.  Up to kZeroCopyBytes (16 MiB) of clients the kernel
// reads the pinned image itself over PCIe in 16-byte loads (no copy call;
// config 2's 7.9 MB: 267 us vs 274 us through DMA, tools/small_agg_bench.py);
// larger rounds go up in ~1 MiB DMAs into cached device rows, each packed
// while the previous one is in flight.  Either way the kernel
// writes the result straight into pinned memory and its last workgroup raises
// a completion word there, which the host spins on: no stream synchronise.
// Same arithmetic as every FedAvg kernel: acc = x_0*w_0; acc = acc + x_i*w_i.

constexpr int64_t kZeroCopyBytes = int64_t(16) << 20;
constexpr int kRoundBlock = 256;

__global__ __launch_bounds__(kRoundBlock) void host_round_kernel(const float* __restrict__ rows, int64_t L, int K,
                                                                 InlW<float> w, float* __restrict__ res,
                                                                 unsigned int* __restrict__ counter,
                                                                 unsigned int* __restrict__ flag, unsigned int seq) {
  // four consecutive elements per lane (L is a multiple of 64): 16-byte
  // loads, 1 KiB per wave instruction, so reads over PCIe travel in full lines
  const int64_t e = (int64_t(blockIdx.x) * kRoundBlock + threadIdx.x) * 4;
  if (e < L) {
    // 8 client loads in flight, the last group predicated: read over PCIe
    // from pinned memory each is a full round trip, so latency, not bytes,
    // is the cost
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int c = 0; c < K; c += 8) {
      float4 x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        x[u] = (c + u < K) ? *reinterpret_cast<const float4*>(rows + int64_t(c + u) * L + e)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (c + u >= K) continue;
        const float wu = w[c + u];
        if (c + u == 0) {
          acc = make_float4(x[u].x * wu, x[u].y * wu, x[u].z * wu, x[u].w * wu);
        } else {
          acc.x = acc.x + x[u].x * wu;
          acc.y = acc.y + x[u].y * wu;
          acc.z = acc.z + x[u].z * wu;
          acc.w = acc.w + x[u].w * wu;
        }
      }
    }
    *reinterpret_cast<float4*>(res + e) = acc;
  }
  // every workgroup's result stores are visible system-wide before it is
  // counted; the last one resets the counter and raises the host's word
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int prev = atomicAdd(counter, 1u);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ---------------------------------------------------------------------------
// One small round of device tensors in one launch (fedagg_device_round_f32).
//
// A GPU server (`using_gpu`) hands FedMLAggOperator.agg device tensors; at
// config 1 (4 clients x 2 keys, 31 KB) the reduction is a few microseconds and
// the pointer-table and weight uploads, output allocation and per-key launches
// around it decide the time.  Here every client pointer, output pointer, key
// length and weight travels in the kernel arguments (no upload at all) and one
// launch covers every key: a workgroup owns 1,024 consecutive elements of one
// key (4 per lane, 16-byte loads), keys looked up by a wave-uniform scan of
// their first-block prefix.  Same arithmetic as every FedAvg kernel:
// acc = x_0*w_0; acc = acc + x_i*w_i; int64 keys as fl32(v) (torch's int64 *
// float promotion) into fp32 outputs.
constexpr int kDevRoundMaxKeys = 16;
constexpr int kDevRoundMaxPtrs = 128;
constexpr int kDevRoundBlock = 256;
constexpr int kDevRoundElems = kDevRoundBlock * 4;

struct DevRoundArgs {
  const void* src[kDevRoundMaxPtrs];  // [T][K]
  float* out[kDevRoundMaxKeys];
  int64_t numel[kDevRoundMaxKeys];
  int64_t block0[kDevRoundMaxKeys + 1];  // first workgroup of key t; block0[T] = grid
  float w[kDevRoundMaxPtrs];
  int32_t code[kDevRoundMaxKeys];
  int32_t T, K;
};

template <class T>
__device__ __forceinline__ float dr_load(const void* p, int64_t e) {
  if constexpr (std::is_same<T, float>::value)
    return reinterpret_cast<const float*>(p)[e];
  else
    return static_cast<float>(reinterpret_cast<const int64_t*>(p)[e]);
}

template <class T>
__device__ __forceinline__ void dr_key(const DevRoundArgs& a, int t, int64_t e, int64_t n) {
  const void* const* src = a.src + t * a.K;
  if (e + 4 <= n && std::is_same<T, float>::value) {
    float4 acc;
    {
      const float4 x = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(src[0]) + e);
      const float w0 = a.w[0];
      acc = make_float4(x.x * w0, x.y * w0, x.z * w0, x.w * w0);
    }
    for (int i = 1; i < a.K; ++i) {
      const float4 x = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(src[i]) + e);
      const float wi = a.w[i];
      acc.x = acc.x + x.x * wi;
      acc.y = acc.y + x.y * wi;
      acc.z = acc.z + x.z * wi;
      acc.w = acc.w + x.w * wi;
    }
    *reinterpret_cast<float4*>(a.out[t] + e) = acc;
    return;
  }
  for (int64_t j = e; j < e + 4 && j < n; ++j) {
    float acc = dr_load<T>(src[0], j) * a.w[0];
    for (int i = 1; i < a.K; ++i) acc = acc + dr_load<T>(src[i], j) * a.w[i];
    a.out[t][j] = acc;
  }
}

__global__ __launch_bounds__(kDevRoundBlock) void device_round_kernel(const DevRoundArgs a) {
  int t = 0;
  while (t + 1 < a.T && int64_t(blockIdx.x) >= a.block0[t + 1]) ++t;  // wave-uniform
  const int64_t e = (int64_t(blockIdx.x) - a.block0[t]) * kDevRoundElems + int64_t(threadIdx.x) * 4;
  const int64_t n = a.numel[t];
  if (e >= n) return;
  if (a.code[t] == FEDAGG_DT_F32)
    dr_key<float>(a, t, e, n);
  else
    dr_key<int64_t>(a, t, e, n);
}

// A persistent pool for the host copies of a round (spawning threads per call
// costs more than a config-2 pack).
class HostPool {
 public:
  static HostPool& get() {
    static HostPool* p = new HostPool(std::max(1u, std::min(8u, std::thread::hardware_concurrency())) - 1);
    return *p;
  }
  int size() const { return int(workers_.size()) + 1; }
  void run(int parts, const std::function<void(int)>& fn) {
    parts = std::max(1, std::min(parts, size()));
    if (parts == 1) {
      fn(0);
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &fn;
      parts_ = parts;
      next_.store(1);
      pending_ = parts - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0 && active_ == 0; });
    job_ = nullptr;
  }

 private:
  explicit HostPool(unsigned n) {
    for (unsigned i = 0; i < n; ++i) std::thread([this] { loop(); }).detach();
    workers_.resize(n);
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (!job_) continue;
      const std::function<void(int)>* fn = job_;
      const int parts = parts_;
      ++active_;
      lk.unlock();
      int done = 0;
      for (int part = next_.fetch_add(1); part < parts; part = next_.fetch_add(1), ++done) (*fn)(part);
      lk.lock();
      pending_ -= done;
      --active_;
      if (pending_ == 0 && active_ == 0) done_cv_.notify_one();
    }
  }
  std::vector<char> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* job_ = nullptr;
  int parts_ = 0, pending_ = 0, active_ = 0;
  std::atomic<int> next_{1};
  uint64_t gen_ = 0;
};

// Buffers of one device, grown on demand and kept (a server runs the same
// round shape every round): the pinned image, the pinned result, the device
// rows of the DMA path, the completion word and the workgroup counter.
struct RoundCtx {
  float* stage = nullptr;
  size_t stage_n = 0;
  float* res = nullptr;
  size_t res_n = 0;
  float* rows = nullptr;
  size_t rows_n = 0;
  unsigned int* flag = nullptr;
  unsigned int* counter = nullptr;
  unsigned int seq = 0;
  hipStream_t own = nullptr;
};
std::mutex g_round_mu;
std::vector<RoundCtx> g_round_ctx;

int grow_pinned(float** p, size_t* have, size_t need) {
  if (*have >= need) return FEDAGG_OK;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *have = 0;
  const size_t n = need + need / 4;
  if (hipHostMalloc(reinterpret_cast<void**>(p), n * sizeof(float), hipHostMallocCoherent | hipHostMallocMapped) !=
      hipSuccess)
    return set_error(FEDAGG_EINVAL, "fedagg_host_round_f32: pinned allocation failed");
  *have = n;
  return FEDAGG_OK;
}

template <class F>
void split_rows(int64_t bytes, int n, const F& fn) {  // fn(i) for i in [0, n), across the pool for big copies
  if (bytes < (int64_t(256) << 10) || n < 2) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  HostPool& pool = HostPool::get();
  const int parts = std::min(pool.size(), n);
  pool.run(parts, [&](int part) {
    for (int i = part; i < n; i += parts) fn(i);
  });
}

// ===========================================================================
// C ABI
// ===========================================================================

// FedAvg fused with a server-optimizer epilogue (SgdEpi / AdamEpi): the tile
// configuration by size, as launch_ws picks it for plain FedAvg.  FUSED_CAP
// selects reduce_fused_kernel (capped at 128 VGPRs for Adam's operands).
template <bool FUSED_CAP, class C, class EPI, class WS>
void launch_fused_cfg(const Seg<OpF32>& s, const EPI& epi, const WS& w, int32_t K, bool aligned, hipStream_t st) {
  const int64_t grid = ((s.numel + 3) / 4 + int64_t(C::BS) * C::V - 1) / (int64_t(C::BS) * C::V);
  const dim3 g{unsigned(grid)}, b{unsigned(C::BS)};
  // The cap only pays on the aligned fast path (the prefetched operands live
  // across the client loop there); the unaligned edge path keeps V*E chains
  // in flight and spills under it, so it runs uncapped.
  if (aligned) {
    if constexpr (FUSED_CAP)
      hipLaunchKernelGGL((reduce_fused_kernel<OpF32, C::U, C::V, C::NT, true, C::BS, EPI, WS>), g, b, 0, st, s, epi, w, K);
    else
      hipLaunchKernelGGL((reduce_kernel<OpF32, C::U, C::V, C::NT, true, C::BS, EPI, WS>), g, b, 0, st, s, epi, w, K);
  } else {
    hipLaunchKernelGGL((reduce_kernel<OpF32, C::U, C::V, C::NT, false, C::BS, EPI, WS>), g, b, 0, st, s, epi, w, K);
  }
}

template <bool FUSED_CAP, class EPI, class WS>
void launch_fused(const Seg<OpF32>& s, const EPI& epi, const WS& w, int32_t K, bool aligned, hipStream_t st) {
  const int64_t blocks = blocks_for<OpF32>(s.numel);
  // A device's shard of a one-process multi-GPU FedOpt round (config 5 over 8
  // GPUs: 16 keys, 524,288 elements) is 128 mid tiles: half the CUs.  The
  // plain FedAvg tiers apply (§6a).
  if (blocks < kSmallBelowBlocks)
    launch_fused_cfg<FUSED_CAP, SmallCfg>(s, epi, w, K, aligned, st);
  else if (blocks < kMid2BelowBlocks)
    launch_fused_cfg<FUSED_CAP, Mid2Cfg>(s, epi, w, K, aligned, st);
  else if (blocks <= kMidUpToBlocks)
    launch_fused_cfg<FUSED_CAP, MidCfg>(s, epi, w, K, aligned, st);
  else
    launch_fused_cfg<FUSED_CAP, Cfg<OpF32>>(s, epi, w, K, aligned, st);
}

template <class OP>
int launch_multi(const void* const* d_src, void* const* d_out, const int64_t* d_numel, const int64_t* d_block_begin,
                 int32_t T, const float* d_w, int32_t K, int64_t total_blocks, hipStream_t st) {
  using C = Cfg<OP>;
  hipLaunchKernelGGL((reduce_multi_kernel<OP, C::U, C::V, C::NT, C::BS>), dim3(unsigned(total_blocks)), dim3(C::BS),
                     0, st, reinterpret_cast<const typename OP::in_t* const*>(d_src),
                     reinterpret_cast<typename OP::out_t* const*>(d_out), d_numel, d_block_begin, T, d_w, K);
  return check_launch("fedagg_wsum_multi");
}
}  // namespace


extern "C" {

int fedagg_wsum_f32(const float* const* d_src, const float* d_w, int32_t K, int64_t N, float* d_out,
                    uint32_t flags, fedagg_stream_t stream) {
  return launch<OpF32>(reinterpret_cast<const void* const*>(d_src), d_w, K, N, d_out, flags, stream,
                       "fedagg_wsum_f32");
}

int fedagg_wsum_rlr_f32(const float* const* d_src, const float* d_w, int32_t K, int64_t N, float threshold,
                        float* d_out, uint32_t flags, fedagg_stream_t stream) {
  const char* name = "fedagg_wsum_rlr_f32";
  if (K < 1 || N < 0) return set_error(FEDAGG_EINVAL, std::string(name) + ": K must be >= 1 and N >= 0");
  if (!d_src || !d_out || !d_w) return set_error(FEDAGG_EINVAL, std::string(name) + ": null pointer");
  if (N == 0) return FEDAGG_OK;
  const Seg<OpF32Rlr> s{d_src, N};
  const RlrEpi epi{d_out, threshold};
  const bool al = (flags & FEDAGG_ALIGNED16) != 0;
  auto st = reinterpret_cast<hipStream_t>(stream);
  if (flags & FEDAGG_HOST_WEIGHTS) {
    InlW<float> iw;
    if (!inline_weights<float>(d_w, K, &iw))
      return set_error(FEDAGG_EINVAL, std::string(name) + ": FEDAGG_HOST_WEIGHTS needs K <= 256");
    return launch_epi<OpF32Rlr>(s, epi, iw, K, al, st, name);
  }
  return launch_epi<OpF32Rlr>(s, epi, PtrW<float>{d_w}, K, al, st, name);
}

int fedagg_wsum_bf16(const uint16_t* const* d_src, const float* d_w, int32_t K, int64_t N, uint16_t* d_out,
                     int32_t acc_mode, uint32_t flags, fedagg_stream_t stream) {
  auto src = reinterpret_cast<const void* const*>(d_src);
  if (acc_mode == FEDAGG_ACC_REFERENCE)
    return launch<OpBF16Ref>(src, d_w, K, N, d_out, flags, stream, "fedagg_wsum_bf16");
  if (acc_mode == FEDAGG_ACC_FP32)
    return launch<OpBF16Acc32>(src, d_w, K, N, d_out, flags, stream, "fedagg_wsum_bf16");
  return set_error(FEDAGG_EINVAL, "fedagg_wsum_bf16: unknown acc_mode");
}

int fedagg_wsum_bf16_f32out(const uint16_t* const* d_src, const float* d_w, int32_t K, int64_t N, float* d_out,
                            uint32_t flags, fedagg_stream_t stream) {
  // The fp32 output pack of 8 bf16 inputs is 32 bytes: the aligned fast path
  // stores two 16-byte halves, so require 32-byte output alignment implicitly
  // via the 16-byte flag (torch's allocator gives 512-byte aligned storage).
  return launch<OpBF16F32Out>(reinterpret_cast<const void* const*>(d_src), d_w, K, N, d_out, flags, stream,
                              "fedagg_wsum_bf16_f32out");
}

int fedagg_wsum_f16(const uint16_t* const* d_src, const float* d_w, int32_t K, int64_t N, uint16_t* d_out,
                    int32_t acc_mode, uint32_t flags, fedagg_stream_t stream) {
  auto src = reinterpret_cast<const void* const*>(d_src);
  if (acc_mode == FEDAGG_ACC_REFERENCE)
    return launch<OpF16Ref>(src, d_w, K, N, d_out, flags, stream, "fedagg_wsum_f16");
  if (acc_mode == FEDAGG_ACC_FP32)
    return launch<OpF16Acc32>(src, d_w, K, N, d_out, flags, stream, "fedagg_wsum_f16");
  return set_error(FEDAGG_EINVAL, "fedagg_wsum_f16: unknown acc_mode");
}

int fedagg_wsum_f64(const double* const* d_src, const double* d_w64, int32_t K, int64_t N, double* d_out,
                    uint32_t flags, fedagg_stream_t stream) {
  return launch<OpF64>(reinterpret_cast<const void* const*>(d_src), d_w64, K, N, d_out, flags, stream,
                       "fedagg_wsum_f64");
}

int fedagg_wsum_i64_f32(const int64_t* const* d_src, const float* d_w, int32_t K, int64_t N, float* d_out,
                        uint32_t flags, fedagg_stream_t stream) {
  return launch<OpI64F32>(reinterpret_cast<const void* const*>(d_src), d_w, K, N, d_out, flags, stream,
                          "fedagg_wsum_i64_f32");
}

int fedagg_sum(int32_t dtype, const void* const* d_src, int32_t K, int64_t N, void* d_out, uint32_t flags,
               fedagg_stream_t stream) {
  switch (dtype) {
    case FEDAGG_DT_F32: return launch<OpSumF32>(d_src, nullptr, K, N, d_out, flags, stream, "fedagg_sum", false);
    case FEDAGG_DT_BF16: return launch<OpSumBF16>(d_src, nullptr, K, N, d_out, flags, stream, "fedagg_sum", false);
    case FEDAGG_DT_F16: return launch<OpSumF16>(d_src, nullptr, K, N, d_out, flags, stream, "fedagg_sum", false);
    case FEDAGG_DT_F64: return launch<OpSumF64>(d_src, nullptr, K, N, d_out, flags, stream, "fedagg_sum", false);
    case FEDAGG_DT_I64: return launch<OpSumI64>(d_src, nullptr, K, N, d_out, flags, stream, "fedagg_sum", false);
    case FEDAGG_DT_I32: return launch<OpSumI32>(d_src, nullptr, K, N, d_out, flags, stream, "fedagg_sum", false);
    default: return set_error(FEDAGG_EINVAL, "fedagg_sum: unsupported dtype");
  }
}

int fedagg_wsum_muldiv(int32_t dtype, const void* const* d_src, const void* d_w, int32_t K, int64_t N, void* d_out,
                       uint32_t flags, fedagg_stream_t stream) {
  const char* name = "fedagg_wsum_muldiv";
  if (K < 1 || N < 0) return set_error(FEDAGG_EINVAL, std::string(name) + ": K must be >= 1 and N >= 0");
  if (!d_src || !d_out || !d_w) return set_error(FEDAGG_EINVAL, std::string(name) + ": null pointer");
  if (flags & FEDAGG_HOST_WEIGHTS) return set_error(FEDAGG_EINVAL, std::string(name) + ": device weights only");
  if (N == 0) return FEDAGG_OK;
  const bool al = (flags & FEDAGG_ALIGNED16) != 0;
  auto st = reinterpret_cast<hipStream_t>(stream);
  auto go = [&](auto op) {
    using OP = decltype(op);
    Seg<OP> seg{reinterpret_cast<const typename OP::in_t* const*>(d_src), N};
    return launch_epi<OP>(seg, StoreEpi<OP>{reinterpret_cast<typename OP::out_t*>(d_out)},
                          PtrW<typename OP::w_t>{reinterpret_cast<const typename OP::w_t*>(d_w)}, K, al, st, name);
  };
  switch (dtype) {
    case FEDAGG_DT_F32: return go(OpF32MulDiv{});
    case FEDAGG_DT_BF16: return go(OpBF16MulDiv{});
    case FEDAGG_DT_F16: return go(OpF16MulDiv{});
    case FEDAGG_DT_F64: return go(OpF64MulDiv{});
    case FEDAGG_DT_I64: return go(OpI64MulDiv{});
    default: return set_error(FEDAGG_EINVAL, std::string(name) + ": unsupported dtype");
  }
}

int64_t fedagg_multi_blocks(int32_t dtype, int64_t numel) {
  if (numel < 0) return -1;
  switch (dtype) {
    case FEDAGG_DT_F32: return blocks_for<OpF32>(numel);
    case FEDAGG_DT_BF16: return blocks_for<OpBF16Ref>(numel);
    case FEDAGG_DT_F16: return blocks_for<OpF16Ref>(numel);
    case FEDAGG_DT_I64: return blocks_for<OpI64F32>(numel);
    default: return -1;
  }
}


int fedagg_wsum_multi(int32_t dtype, int32_t acc_mode, const void* const* d_src, void* const* d_out,
                      const int64_t* d_numel, const int64_t* d_block_begin, int32_t T, const float* d_w, int32_t K,
                      int64_t total_blocks, fedagg_stream_t stream) {
  if (K < 1 || T < 1 || total_blocks < 0) return set_error(FEDAGG_EINVAL, "fedagg_wsum_multi: bad sizes");
  if (!d_src || !d_out || !d_numel || !d_block_begin || !d_w)
    return set_error(FEDAGG_EINVAL, "fedagg_wsum_multi: null pointer");
  if (acc_mode != FEDAGG_ACC_REFERENCE && acc_mode != FEDAGG_ACC_FP32)
    return set_error(FEDAGG_EINVAL, "fedagg_wsum_multi: unknown acc_mode");
  if (total_blocks == 0) return FEDAGG_OK;
  if (total_blocks > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, "fedagg_wsum_multi: too many blocks");
  auto st = reinterpret_cast<hipStream_t>(stream);
  const bool ref = acc_mode == FEDAGG_ACC_REFERENCE;
  switch (dtype) {
    case FEDAGG_DT_F32: return launch_multi<OpF32>(d_src, d_out, d_numel, d_block_begin, T, d_w, K, total_blocks, st);
    case FEDAGG_DT_BF16:
      return ref ? launch_multi<OpBF16Ref>(d_src, d_out, d_numel, d_block_begin, T, d_w, K, total_blocks, st)
                 : launch_multi<OpBF16Acc32>(d_src, d_out, d_numel, d_block_begin, T, d_w, K, total_blocks, st);
    case FEDAGG_DT_F16:
      return ref ? launch_multi<OpF16Ref>(d_src, d_out, d_numel, d_block_begin, T, d_w, K, total_blocks, st)
                 : launch_multi<OpF16Acc32>(d_src, d_out, d_numel, d_block_begin, T, d_w, K, total_blocks, st);
    case FEDAGG_DT_I64:
      return launch_multi<OpI64F32>(d_src, d_out, d_numel, d_block_begin, T, d_w, K, total_blocks, st);
    default: return set_error(FEDAGG_EINVAL, "fedagg_wsum_multi: unsupported dtype");
  }
}

int fedagg_wsum_multi_f32(const float* const* d_src, float* const* d_out, const int64_t* d_numel,
                          const int64_t* d_block_begin, int32_t T, const float* d_w, int32_t K,
                          int64_t total_blocks, fedagg_stream_t stream) {
  return fedagg_wsum_multi(FEDAGG_DT_F32, FEDAGG_ACC_REFERENCE, reinterpret_cast<const void* const*>(d_src),
                           reinterpret_cast<void* const*>(d_out), d_numel, d_block_begin, T, d_w, K, total_blocks,
                           stream);
}

int fedagg_fedopt_sgd_f32(float* d_param, float* d_mom, const float* d_avg, int64_t N, float lr, float momentum,
                          int32_t first_step, fedagg_stream_t stream) {
  if (N < 0 || !d_param || !d_avg) return set_error(FEDAGG_EINVAL, "fedagg_fedopt_sgd_f32: bad argument");
  if (N == 0) return FEDAGG_OK;
  const int64_t want = (N + kBlock - 1) / kBlock;
  const unsigned grid = unsigned(want < 8192 ? want : 8192);
  hipLaunchKernelGGL(fedopt_sgd_kernel, dim3(grid), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream), d_param,
                     momentum != 0.0f ? d_mom : nullptr, d_avg, N, -lr, momentum, first_step);
  return check_launch("fedagg_fedopt_sgd_f32");
}

int fedagg_wsum_fedopt_sgd_f32(const float* const* d_src, const float* d_w, int32_t K, int64_t N, float* d_param,
                               float* d_mom, float lr, float momentum, int32_t first_step, uint32_t flags,
                               fedagg_stream_t stream) {
  if (K < 1 || N < 0) return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_sgd_f32: K must be >= 1 and N >= 0");
  if (!d_src || !d_w || !d_param || (momentum != 0.0f && !d_mom))
    return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_sgd_f32: null pointer");
  if (N == 0) return FEDAGG_OK;
  const int64_t grid = blocks_for<OpF32>(N);
  if (grid > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_sgd_f32: N too large");
  Seg<OpF32> s{d_src, N};
  SgdEpi epi{d_param, momentum != 0.0f ? d_mom : nullptr, -lr, momentum, first_step};
  auto st = reinterpret_cast<hipStream_t>(stream);
  const bool aligned = (flags & FEDAGG_ALIGNED16) != 0;
  if (flags & FEDAGG_HOST_WEIGHTS) {
    InlW<float> iw;
    if (!inline_weights<float>(d_w, K, &iw))
      return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_sgd_f32: FEDAGG_HOST_WEIGHTS needs K <= 256");
    launch_fused<true>(s, epi, iw, K, aligned, st);
  } else {
    launch_fused<true>(s, epi, PtrW<float>{d_w}, K, aligned, st);
  }
  return check_launch("fedagg_wsum_fedopt_sgd_f32");
}

int fedagg_adam_scalars(double lr, double beta1, double beta2, double eps, int64_t step, float* out6) {
  if (!out6 || step < 1) return set_error(FEDAGG_EINVAL, "fedagg_adam_scalars: step must be >= 1");
  // the double-precision scalar chain of torch.optim.adam._single_tensor_adam;
  // Python's ** is C pow(), so bias_correction2 ** 0.5 is pow(x, 0.5), not sqrt
  const double t = double(step);
  const double bc1 = 1.0 - std::pow(beta1, t);
  const double bc2 = 1.0 - std::pow(beta2, t);
  const double step_size = lr / bc1;
  out6[0] = float(1.0 - beta1);         // lerp_ weight
  out6[1] = float(beta2);               // mul_
  out6[2] = float(1.0 - beta2);         // addcmul_ value
  out6[3] = float(std::pow(bc2, 0.5));  // bias_correction2_sqrt
  out6[4] = float(eps);                 // add_
  out6[5] = float(-step_size);          // addcdiv_ value
  return FEDAGG_OK;
}

int fedagg_wsum_fedopt_adam_f32(const float* const* d_src, const float* d_w, int32_t K, int64_t N, float* d_param,
                                float* d_exp_avg, float* d_exp_avg_sq, const float* scalars6, int32_t first_step,
                                uint32_t flags, fedagg_stream_t stream) {
  if (K < 1 || N < 0) return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_adam_f32: K must be >= 1 and N >= 0");
  if (!d_src || !d_w || !d_param || !d_exp_avg || !d_exp_avg_sq || !scalars6)
    return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_adam_f32: null pointer");
  if (N == 0) return FEDAGG_OK;
  const int64_t grid = blocks_for<OpF32>(N);
  if (grid > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_adam_f32: N too large");
  Seg<OpF32> s{d_src, N};
  AdamEpi epi{d_param, d_exp_avg, d_exp_avg_sq, scalars6[0], scalars6[1], scalars6[2],
              scalars6[3], scalars6[4], scalars6[5], first_step};
  auto st = reinterpret_cast<hipStream_t>(stream);
  const bool aligned = (flags & FEDAGG_ALIGNED16) != 0;
  if (flags & FEDAGG_HOST_WEIGHTS) {
    InlW<float> iw;
    if (!inline_weights<float>(d_w, K, &iw))
      return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_adam_f32: FEDAGG_HOST_WEIGHTS needs K <= 256");
    launch_fused<true>(s, epi, iw, K, aligned, st);
  } else {
    launch_fused<true>(s, epi, PtrW<float>{d_w}, K, aligned, st);
  }
  return check_launch("fedagg_wsum_fedopt_adam_f32");
}

int fedagg_wsum_fedopt_adagrad_f32(const float* const* d_src, const float* d_w, int32_t K, int64_t N, float* d_param,
                                   float* d_sum, float clr, float eps, uint32_t flags, fedagg_stream_t stream) {
  if (K < 1 || N < 0) return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_adagrad_f32: K must be >= 1 and N >= 0");
  if (!d_src || !d_w || !d_param || !d_sum)
    return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_adagrad_f32: null pointer");
  if (N == 0) return FEDAGG_OK;
  const int64_t grid = blocks_for<OpF32>(N);
  if (grid > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_adagrad_f32: N too large");
  Seg<OpF32> s{d_src, N};
  AdagradEpi epi{d_param, d_sum, -clr, eps};
  auto st = reinterpret_cast<hipStream_t>(stream);
  const bool aligned = (flags & FEDAGG_ALIGNED16) != 0;
  if (flags & FEDAGG_HOST_WEIGHTS) {
    InlW<float> iw;
    if (!inline_weights<float>(d_w, K, &iw))
      return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_adagrad_f32: FEDAGG_HOST_WEIGHTS needs K <= 256");
    launch_fused<false>(s, epi, iw, K, aligned, st);
  } else {
    launch_fused<false>(s, epi, PtrW<float>{d_w}, K, aligned, st);
  }
  return check_launch("fedagg_wsum_fedopt_adagrad_f32");
}

int fedagg_wsum_fedopt_adamw_f32(const float* const* d_src, const float* d_w, int32_t K, int64_t N, float* d_param,
                                 float* d_exp_avg, float* d_exp_avg_sq, const float* scalars6, float decay,
                                 int32_t first_step, uint32_t flags, fedagg_stream_t stream) {
  if (K < 1 || N < 0) return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_adamw_f32: K must be >= 1 and N >= 0");
  if (!d_src || !d_w || !d_param || !d_exp_avg || !d_exp_avg_sq || !scalars6)
    return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_adamw_f32: null pointer");
  if (N == 0) return FEDAGG_OK;
  const int64_t grid = blocks_for<OpF32>(N);
  if (grid > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_adamw_f32: N too large");
  Seg<OpF32> s{d_src, N};
  AdamEpi epi{d_param, d_exp_avg, d_exp_avg_sq, scalars6[0], scalars6[1], scalars6[2],
              scalars6[3], scalars6[4], scalars6[5], first_step, decay, 1};
  auto st = reinterpret_cast<hipStream_t>(stream);
  const bool aligned = (flags & FEDAGG_ALIGNED16) != 0;
  if (flags & FEDAGG_HOST_WEIGHTS) {
    InlW<float> iw;
    if (!inline_weights<float>(d_w, K, &iw))
      return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_adamw_f32: FEDAGG_HOST_WEIGHTS needs K <= 256");
    launch_fused<true>(s, epi, iw, K, aligned, st);
  } else {
    launch_fused<true>(s, epi, PtrW<float>{d_w}, K, aligned, st);
  }
  return check_launch("fedagg_wsum_fedopt_adamw_f32");
}

int fedagg_wsum_fedopt_rmsprop_f32(const float* const* d_src, const float* d_w, int32_t K, int64_t N,
                                   float* d_param, float* d_square_avg, float lr, double alpha, float eps,
                                   uint32_t flags, fedagg_stream_t stream) {
  if (K < 1 || N < 0) return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_rmsprop_f32: K must be >= 1 and N >= 0");
  if (!d_src || !d_w || !d_param || !d_square_avg)
    return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_rmsprop_f32: null pointer");
  if (N == 0) return FEDAGG_OK;
  const int64_t grid = blocks_for<OpF32>(N);
  if (grid > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_rmsprop_f32: N too large");
  Seg<OpF32> s{d_src, N};
  // alpha and 1 - alpha are Python floats (doubles) that torch's CPU kernels
  // round to fp32 each
  AdagradEpi epi{d_param, d_square_avg, -lr, eps, float(alpha), float(1.0 - alpha)};
  auto st = reinterpret_cast<hipStream_t>(stream);
  const bool aligned = (flags & FEDAGG_ALIGNED16) != 0;
  if (flags & FEDAGG_HOST_WEIGHTS) {
    InlW<float> iw;
    if (!inline_weights<float>(d_w, K, &iw))
      return set_error(FEDAGG_EINVAL, "fedagg_wsum_fedopt_rmsprop_f32: FEDAGG_HOST_WEIGHTS needs K <= 256");
    launch_fused<false>(s, epi, iw, K, aligned, st);
  } else {
    launch_fused<false>(s, epi, PtrW<float>{d_w}, K, aligned, st);
  }
  return check_launch("fedagg_wsum_fedopt_rmsprop_f32");
}

int fedagg_optrepo_scalars(int32_t opt, double lr, int64_t step, float* carry2, float* out9) {
  if (!out9 || step < 1) return set_error(FEDAGG_EINVAL, "fedagg_optrepo_scalars: step must be >= 1");
  for (int i = 0; i < 9; ++i) out9[i] = 0.0f;
  // torch's double-precision scalar chains (Python's ** is C pow()); every
  // value a CPU kernel receives as a Python float is rounded to fp32 here
  const double t = double(step);
  const double b1 = 0.9, b2 = 0.999;
  switch (opt) {
    case kOptAdamax: {
      const double clr = lr / (1.0 - std::pow(b1, t));
      out9[0] = float(1.0 - b1); out9[1] = float(b2); out9[2] = float(1e-8); out9[3] = float(-clr);
      return FEDAGG_OK;
    }
    case kOptNAdam: {
      if (!carry2) return set_error(FEDAGG_EINVAL, "fedagg_optrepo_scalars: NAdam needs carry2 (mu_product)");
      const double md = 4e-3;
      const double mu = b1 * (1.0 - 0.5 * std::pow(0.96, t * md));
      const double mu_next = b1 * (1.0 - 0.5 * std::pow(0.96, (t + 1.0) * md));
      carry2[0] = carry2[0] * float(mu);  // mu_product *= mu: an fp32 state tensor
      const double mp = double(carry2[0]);
      const double mp_next = mp * mu_next;
      out9[0] = float(1.0 - b1); out9[1] = float(b2); out9[2] = float(1.0 - b2);
      out9[3] = float(1.0 - std::pow(b2, t)); out9[4] = float(1e-8);
      out9[5] = float(-lr * (1.0 - mu) / (1.0 - mp));
      out9[6] = float(-lr * mu_next / (1.0 - mp_next));
      return FEDAGG_OK;
    }
    case kOptRAdam: {
      const double bc1 = 1.0 - std::pow(b1, t), bc2 = 1.0 - std::pow(b2, t);
      const double rho_inf = 2.0 / (1.0 - b2) - 1.0;
      const double rho_t = rho_inf - 2.0 * t * std::pow(b2, t) / bc2;
      out9[0] = float(1.0 - b1); out9[1] = float(b2); out9[2] = float(1.0 - b2);
      out9[3] = float(bc1); out9[4] = float(lr); out9[6] = float(1e-8);
      if (rho_t > 5.0) {
        out9[5] = 1.0f;
        out9[7] = float(std::pow(bc2, 0.5));
        out9[8] = float(std::pow((rho_t - 4.0) * (rho_t - 2.0) * rho_inf / ((rho_inf - 4.0) * (rho_inf - 2.0) * rho_t),
                                 0.5));
      }
      return FEDAGG_OK;
    }
    case kOptAdadelta:
      out9[0] = float(0.9); out9[1] = float(1.0 - 0.9); out9[2] = float(1e-6); out9[3] = float(-lr);
      return FEDAGG_OK;
    case kOptASGD: {
      if (!carry2) return set_error(FEDAGG_EINVAL, "fedagg_optrepo_scalars: ASGD needs carry2 (eta, mu)");
      const double lambd = 1e-4, alpha = 0.75, t0 = 1e6;
      const double eta = double(carry2[0]);
      out9[0] = float(1.0 - lambd * eta); out9[1] = float(-eta); out9[2] = carry2[1];
      out9[3] = carry2[1] == 1.0f ? 1.0f : 0.0f;
      carry2[0] = float(lr / std::pow(1.0 + lambd * lr * t, alpha));  // eta.copy_(...), after the step
      carry2[1] = float(1.0 / std::max(1.0, t - t0));
      return FEDAGG_OK;
    }
    case kOptRprop:
      out9[0] = float(1.2); out9[1] = float(0.5); out9[2] = float(1e-6); out9[3] = float(50.0);
      return FEDAGG_OK;
    default:
      return set_error(FEDAGG_EINVAL, "fedagg_optrepo_scalars: unknown optimizer code");
  }
}

int fedagg_wsum_fedopt_optrepo_f32(int32_t opt, const float* const* d_src, const float* d_w, int32_t K, int64_t N,
                                   float* d_param, float* d_state0, float* d_state1, const float* scalars9,
                                   uint32_t flags, fedagg_stream_t stream) {
  const char* name = "fedagg_wsum_fedopt_optrepo_f32";
  if (K < 1 || N < 0) return set_error(FEDAGG_EINVAL, std::string(name) + ": K must be >= 1 and N >= 0");
  if (opt < kOptAdamax || opt > kOptRprop) return set_error(FEDAGG_EINVAL, std::string(name) + ": unknown optimizer");
  if (!d_src || !d_w || !d_param || !d_state0 || (opt != kOptASGD && !d_state1) || !scalars9)
    return set_error(FEDAGG_EINVAL, std::string(name) + ": null pointer");
  if (N == 0) return FEDAGG_OK;
  if (blocks_for<OpF32>(N) > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, std::string(name) + ": N too large");
  const Seg<OpF32> s{d_src, N};
  auto st = reinterpret_cast<hipStream_t>(stream);
  const bool aligned = (flags & FEDAGG_ALIGNED16) != 0;
  InlW<float> iw;
  const bool host_w = (flags & FEDAGG_HOST_WEIGHTS) != 0;
  if (host_w && !inline_weights<float>(d_w, K, &iw))
    return set_error(FEDAGG_EINVAL, std::string(name) + ": FEDAGG_HOST_WEIGHTS needs K <= 256");
  auto run = [&](auto epi) {
    for (int i = 0; i < 9; ++i) epi.k[i] = scalars9[i];
    if (host_w)
      launch_fused<true>(s, epi, iw, K, aligned, st);
    else
      launch_fused<true>(s, epi, PtrW<float>{d_w}, K, aligned, st);
  };
  switch (opt) {
    case kOptAdamax: run(OptRepoEpi<kOptAdamax>{d_param, d_state0, d_state1, {}}); break;
    case kOptNAdam: run(OptRepoEpi<kOptNAdam>{d_param, d_state0, d_state1, {}}); break;
    case kOptRAdam: run(OptRepoEpi<kOptRAdam>{d_param, d_state0, d_state1, {}}); break;
    case kOptAdadelta: run(OptRepoEpi<kOptAdadelta>{d_param, d_state0, d_state1, {}}); break;
    case kOptASGD: run(OptRepoEpi<kOptASGD>{d_param, d_state0, d_state1, {}}); break;
    default: run(OptRepoEpi<kOptRprop>{d_param, d_state0, d_state1, {}}); break;
  }
  return check_launch(name);
}

int fedagg_wsum_fedopt_batch(const fedagg_fedopt_launch* launches, int32_t n) {
  const char* name = "fedagg_wsum_fedopt_batch";
  if (n < 0 || (n > 0 && !launches)) return set_error(FEDAGG_EINVAL, std::string(name) + ": bad argument");
  int cur = -1;
  if (n && hipGetDevice(&cur) != hipSuccess) return set_error(FEDAGG_EINVAL, std::string(name) + ": no device");
  int dev = cur, rc = FEDAGG_OK;
  for (int32_t i = 0; i < n && rc == FEDAGG_OK; ++i) {
    const fedagg_fedopt_launch& l = launches[i];
    if (l.device != dev) {
      if (hipSetDevice(l.device) != hipSuccess) {
        rc = set_error(FEDAGG_EINVAL, std::string(name) + ": bad device ordinal");
        break;
      }
      dev = l.device;
    }
    switch (l.opt) {
      case FEDAGG_FEDOPT_AVG:
        switch (l.dtype) {
          case FEDAGG_DT_F32:
            rc = fedagg_wsum_f32(l.d_src, l.weights, l.K, l.N, l.d_param, l.flags, l.stream);
            break;
          case FEDAGG_DT_BF16:
            rc = fedagg_wsum_bf16(reinterpret_cast<const uint16_t* const*>(l.d_src), l.weights, l.K, l.N,
                                  reinterpret_cast<uint16_t*>(l.d_param), l.acc_mode, l.flags, l.stream);
            break;
          case FEDAGG_DT_F16:
            rc = fedagg_wsum_f16(reinterpret_cast<const uint16_t* const*>(l.d_src), l.weights, l.K, l.N,
                                 reinterpret_cast<uint16_t*>(l.d_param), l.acc_mode, l.flags, l.stream);
            break;
          case FEDAGG_DT_F64:
            rc = fedagg_wsum_f64(reinterpret_cast<const double* const*>(l.d_src),
                                 reinterpret_cast<const double*>(l.weights), l.K, l.N,
                                 reinterpret_cast<double*>(l.d_param), l.flags, l.stream);
            break;
          case FEDAGG_DT_I64:
            rc = fedagg_wsum_i64_f32(reinterpret_cast<const int64_t* const*>(l.d_src), l.weights, l.K, l.N,
                                     l.d_param, l.flags, l.stream);
            break;
          default:
            rc = set_error(FEDAGG_EINVAL, std::string(name) + ": FEDAGG_FEDOPT_AVG dtype");
        }
        break;
      case FEDAGG_FEDOPT_SGD:
        rc = fedagg_wsum_fedopt_sgd_f32(l.d_src, l.weights, l.K, l.N, l.d_param, l.d_state0, l.lr, l.momentum,
                                        l.first_step, l.flags, l.stream);
        break;
      case FEDAGG_FEDOPT_ADAM:
        rc = fedagg_wsum_fedopt_adam_f32(l.d_src, l.weights, l.K, l.N, l.d_param, l.d_state0, l.d_state1, l.scalars,
                                         l.first_step, l.flags, l.stream);
        break;
      case FEDAGG_FEDOPT_ADAMW:
        rc = fedagg_wsum_fedopt_adamw_f32(l.d_src, l.weights, l.K, l.N, l.d_param, l.d_state0, l.d_state1, l.scalars,
                                          l.decay, l.first_step, l.flags, l.stream);
        break;
      case FEDAGG_FEDOPT_ADAGRAD:
        rc = fedagg_wsum_fedopt_adagrad_f32(l.d_src, l.weights, l.K, l.N, l.d_param, l.d_state0, l.lr, l.eps, l.flags,
                                            l.stream);
        break;
      case FEDAGG_FEDOPT_RMSPROP:
        rc = fedagg_wsum_fedopt_rmsprop_f32(l.d_src, l.weights, l.K, l.N, l.d_param, l.d_state0, l.lr, l.alpha, l.eps,
                                            l.flags, l.stream);
        break;
      default:
        if (l.opt >= kOptAdamax && l.opt <= kOptRprop)
          rc = fedagg_wsum_fedopt_optrepo_f32(l.opt, l.d_src, l.weights, l.K, l.N, l.d_param, l.d_state0, l.d_state1,
                                              l.scalars, l.flags, l.stream);
        else
          rc = set_error(FEDAGG_EINVAL, std::string(name) + ": unknown opt code");
    }
  }
  if (dev != cur) (void)hipSetDevice(cur);
  return rc;
}

int fedagg_round_f32(int32_t dtype, const float* d_in, int64_t N, void* d_out, fedagg_stream_t stream) {
  if (N < 0 || (N > 0 && (!d_in || !d_out))) return set_error(FEDAGG_EINVAL, "fedagg_round_f32: bad argument");
  if (dtype != FEDAGG_DT_BF16 && dtype != FEDAGG_DT_F16)
    return set_error(FEDAGG_EINVAL, "fedagg_round_f32: dtype must be FEDAGG_DT_BF16 or FEDAGG_DT_F16");
  if (N == 0) return FEDAGG_OK;
  const int64_t want = (N + kBlock - 1) / kBlock;
  const unsigned grid = unsigned(want < 8192 ? want : 8192);
  auto st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == FEDAGG_DT_BF16)
    hipLaunchKernelGGL(round_f32_kernel<true>, dim3(grid), dim3(kBlock), 0, st, d_in, (uint16_t*)d_out, N);
  else
    hipLaunchKernelGGL(round_f32_kernel<false>, dim3(grid), dim3(kBlock), 0, st, d_in, (uint16_t*)d_out, N);
  return check_launch("fedagg_round_f32");
}

int fedagg_sum_mod_i64(const int64_t* const* d_src, int32_t K, int64_t N, int64_t p, int64_t* d_out,
                       uint32_t flags, fedagg_stream_t stream) {
  if (K < 1 || N < 0) return set_error(FEDAGG_EINVAL, "fedagg_sum_mod_i64: K must be >= 1 and N >= 0");
  if (p <= 0) return set_error(FEDAGG_EINVAL, "fedagg_sum_mod_i64: the prime must be positive");
  if (!d_src || !d_out) return set_error(FEDAGG_EINVAL, "fedagg_sum_mod_i64: null pointer");
  if (N == 0) return FEDAGG_OK;
  Seg<OpSumModI64> s{d_src, N};
  return launch_epi<OpSumModI64>(s, StoreEpi<OpSumModI64>{d_out}, ConstW<int64_t>{p}, K,
                                 (flags & FEDAGG_ALIGNED16) != 0, reinterpret_cast<hipStream_t>(stream),
                                 "fedagg_sum_mod_i64");
}

int fedagg_lsa_reconstruct_f32(const int64_t* const* d_src, int32_t K, int64_t N, const int64_t* d_mask, int64_t p,
                               int32_t q_bits, float w, float* d_out, uint32_t flags, fedagg_stream_t stream) {
  if (K < 1 || N < 0) return set_error(FEDAGG_EINVAL, "fedagg_lsa_reconstruct_f32: K must be >= 1 and N >= 0");
  if (p <= 0 || q_bits < 0 || q_bits > 62)
    return set_error(FEDAGG_EINVAL, "fedagg_lsa_reconstruct_f32: need p > 0 and 0 <= q_bits <= 62");
  if (!d_src || !d_mask || !d_out) return set_error(FEDAGG_EINVAL, "fedagg_lsa_reconstruct_f32: null pointer");
  if (N == 0) return FEDAGG_OK;
  Seg<OpWrapSumI64> s{d_src, N};
  LsaEpi epi{d_mask, d_out, p, ldexp(1.0, -q_bits), w};
  return launch_epi<OpWrapSumI64>(s, epi, ConstW<int64_t>{0}, K, (flags & FEDAGG_ALIGNED16) != 0,
                                  reinterpret_cast<hipStream_t>(stream), "fedagg_lsa_reconstruct_f32");
}


int fedagg_host_pack(void* dst, const void* const* srcs, const int64_t* dst_offs, const int64_t* nbytes, int32_t n,
                     int32_t threads) {
  if (int rc = check_ranges(n, dst, srcs, dst_offs, nbytes, "fedagg_host_pack")) return rc;
  parallel_ranges(
      n, nbytes, threads, [&](int32_t i) { return static_cast<const char*>(srcs[i]); },
      [&](int32_t i) { return static_cast<char*>(dst) + dst_offs[i]; });
  return FEDAGG_OK;
}

int fedagg_host_gather(void* const* dsts, const void* const* srcs, const int64_t* nbytes, int32_t n,
                       int32_t threads) {
  if (n < 0 || (n > 0 && (!dsts || !srcs || !nbytes))) return set_error(FEDAGG_EINVAL, "fedagg_host_gather: bad argument");
  for (int32_t i = 0; i < n; ++i)
    if (nbytes[i] < 0 || (nbytes[i] > 0 && (!dsts[i] || !srcs[i])))
      return set_error(FEDAGG_EINVAL, "fedagg_host_gather: negative size or null pointer");
  parallel_ranges(
      n, nbytes, threads, [&](int32_t i) { return static_cast<const char*>(srcs[i]); },
      [&](int32_t i) { return static_cast<char*>(dsts[i]); });
  return FEDAGG_OK;
}

int fedagg_host_unpack(const void* src, void* const* dsts, const int64_t* src_offs, const int64_t* nbytes, int32_t n,
                       int32_t threads) {
  if (int rc = check_ranges(n, src, dsts, src_offs, nbytes, "fedagg_host_unpack")) return rc;
  parallel_ranges(
      n, nbytes, threads, [&](int32_t i) { return static_cast<const char*>(src) + src_offs[i]; },
      [&](int32_t i) { return static_cast<char*>(dsts[i]); });
  return FEDAGG_OK;
}

int fedagg_device_round_f32(const void* const* d_src, const int32_t* codes, const int64_t* numels, int32_t T,
                            int32_t K, const float* weights, void* const* d_out, fedagg_stream_t stream) {
  const char* name = "fedagg_device_round_f32";
  if (T < 1 || K < 1 || T > kDevRoundMaxKeys || int64_t(T) * K > kDevRoundMaxPtrs || !d_src || !codes || !numels ||
      !weights || !d_out)
    return set_error(FEDAGG_EINVAL, std::string(name) + ": bad argument (T <= 16 keys, T*K <= 128 pointers)");
  DevRoundArgs a;
  a.T = T;
  a.K = K;
  int64_t blocks = 0;
  for (int t = 0; t < T; ++t) {
    if (codes[t] != FEDAGG_DT_F32 && codes[t] != FEDAGG_DT_I64)
      return set_error(FEDAGG_EINVAL, std::string(name) + ": keys must be fp32 or int64");
    if (numels[t] < 0) return set_error(FEDAGG_EINVAL, std::string(name) + ": negative numel");
    for (int i = 0; i < K; ++i) {
      a.src[t * K + i] = d_src[size_t(t) * K + i];
      if (numels[t] && (!a.src[t * K + i] || (reinterpret_cast<uintptr_t>(a.src[t * K + i]) & 15)))
        return set_error(FEDAGG_EINVAL, std::string(name) + ": client pointers must be 16-byte aligned");
    }
    a.out[t] = static_cast<float*>(d_out[t]);
    if (numels[t] && (!a.out[t] || (reinterpret_cast<uintptr_t>(a.out[t]) & 15)))
      return set_error(FEDAGG_EINVAL, std::string(name) + ": outputs must be 16-byte aligned");
    a.numel[t] = numels[t];
    a.code[t] = codes[t];
    a.block0[t] = blocks;
    blocks += (numels[t] + kDevRoundElems - 1) / kDevRoundElems;
  }
  a.block0[T] = blocks;
  for (int i = 0; i < K; ++i) a.w[i] = weights[i];
  if (blocks == 0) return FEDAGG_OK;
  if (blocks > 0x7fffffffLL) return set_error(FEDAGG_EINVAL, std::string(name) + ": round too large");
  hipLaunchKernelGGL(device_round_kernel, dim3(unsigned(blocks)), dim3(kDevRoundBlock), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  return check_launch(name);
}

int fedagg_host_round_f32(const void* const* h_src, const int32_t* codes, const int64_t* numels, int32_t T,
                          int32_t K, const float* weights, void* const* h_out, fedagg_stream_t stream) {
  if (K < 1 || K > kInlineK || T < 0 || (T && (!h_src || !codes || !numels || !h_out)) || !weights)
    return set_error(FEDAGG_EINVAL, "fedagg_host_round_f32: bad argument (1 <= K <= 256)");
  std::vector<int64_t> off(size_t(T) + 1);
  int64_t L = 0;
  for (int32_t t = 0; t < T; ++t) {
    if (codes[t] != FEDAGG_DT_F32 && codes[t] != FEDAGG_DT_I64)
      return set_error(FEDAGG_EINVAL, "fedagg_host_round_f32: keys must be fp32 or int64");
    if (numels[t] < 0) return set_error(FEDAGG_EINVAL, "fedagg_host_round_f32: negative numel");
    off[t] = L;
    L = (L + numels[t] + 3) / 4 * 4;  // next key 16-byte aligned
  }
  if (L == 0) return FEDAGG_OK;
  L = (L + 63) / 64 * 64;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return set_error(FEDAGG_EINVAL, "fedagg_host_round_f32: no device");
  std::lock_guard<std::mutex> lock(g_round_mu);
  if (g_round_ctx.size() <= size_t(dev)) g_round_ctx.resize(size_t(dev) + 1);
  RoundCtx& cx = g_round_ctx[size_t(dev)];
  const int64_t elems = int64_t(K) * L, bytes = elems * 4;
  static const int64_t zc_max = [] {  // FEDAGG_ZERO_COPY_MAX: tuning override (tools/small_agg_bench.py)
    const char* v = getenv("FEDAGG_ZERO_COPY_MAX");
    return v ? int64_t(atoll(v)) : kZeroCopyBytes;
  }();
  const bool zero_copy = bytes <= zc_max;
  if (int rc = grow_pinned(&cx.stage, &cx.stage_n, size_t(elems))) return rc;
  if (int rc = grow_pinned(&cx.res, &cx.res_n, size_t(L))) return rc;
  if (!cx.flag) {
    if (hipHostMalloc(reinterpret_cast<void**>(&cx.flag), 64, hipHostMallocCoherent | hipHostMallocMapped) !=
            hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&cx.counter), 64) != hipSuccess ||
        hipMemset(cx.counter, 0, 64) != hipSuccess)
      return set_error(FEDAGG_EINVAL, "fedagg_host_round_f32: allocation failed");
    __atomic_store_n(cx.flag, 0u, __ATOMIC_RELEASE);
  }
  if (!zero_copy && cx.rows_n < size_t(elems)) {
    if (cx.rows) (void)hipFree(cx.rows);
    cx.rows = nullptr;
    cx.rows_n = 0;
    if (hipMalloc(reinterpret_cast<void**>(&cx.rows), size_t(elems) * 4) != hipSuccess)
      return set_error(FEDAGG_EINVAL, "fedagg_host_round_f32: device allocation failed");
    cx.rows_n = size_t(elems);
  }
  // pack: client i's key t goes to stage[i][off[t]] (int64 keys as fl32(v),
  // the reference's int64 * float promotion)
  auto pack = [&](int i0, int i1) {
    split_rows(int64_t(i1 - i0) * L * 4, i1 - i0, [&](int ii) {
      const int i = i0 + ii;
      float* row = cx.stage + int64_t(i) * L;
      for (int32_t t = 0; t < T; ++t) {
        const void* src = h_src[size_t(t) * K + size_t(i)];
        if (codes[t] == FEDAGG_DT_F32) {
          memcpy(row + off[t], src, size_t(numels[t]) * 4);
        } else {
          const int64_t* v = static_cast<const int64_t*>(src);
          for (int64_t j = 0; j < numels[t]; ++j) row[off[t] + j] = static_cast<float>(v[j]);
        }
      }
    });
  };
  InlW<float> iw;
  for (int i = 0; i < K; ++i) iw.v[i] = weights[i];
  // no stream given: the library's own non-blocking stream (host inputs and
  // outputs; nothing on the caller's streams to order against)
  if (!stream) {
    if (!cx.own) {
      if (hipStreamCreateWithFlags(&cx.own, hipStreamNonBlocking) != hipSuccess)
        return set_error(FEDAGG_EINVAL, "fedagg_host_round_f32: stream creation failed");
    }
    stream = cx.own;
  }
  auto st = reinterpret_cast<hipStream_t>(stream);
  const float* rows = nullptr;
  float* res_d = nullptr;
  unsigned int* flag_d = nullptr;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&res_d), cx.res, 0) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&flag_d), cx.flag, 0) != hipSuccess)
    return set_error(FEDAGG_EINVAL, "fedagg_host_round_f32: pinned memory not device-mapped");
  if (zero_copy) {
    pack(0, K);
    float* stage_d = nullptr;
    if (hipHostGetDevicePointer(reinterpret_cast<void**>(&stage_d), cx.stage, 0) != hipSuccess)
      return set_error(FEDAGG_EINVAL, "fedagg_host_round_f32: pinned memory not device-mapped");
    rows = stage_d;
  } else {
    // ~1 MiB of clients per DMA: packing the next group overlaps the copy of
    // this one
    const int per = int(std::max<int64_t>(1, (int64_t(1) << 20) / (L * 4)));
    for (int i0 = 0; i0 < K; i0 += per) {
      const int i1 = std::min<int>(K, i0 + per);
      pack(i0, i1);
      if (hipMemcpyAsync(cx.rows + int64_t(i0) * L, cx.stage + int64_t(i0) * L, size_t(int64_t(i1 - i0) * L * 4),
                         hipMemcpyHostToDevice, st) != hipSuccess)
        return check_launch("fedagg_host_round_f32 (H2D)");
    }
    rows = cx.rows;
  }
  const unsigned int seq = ++cx.seq == 0 ? ++cx.seq : cx.seq;  // never 0, the word's initial value
  const unsigned grid = unsigned((L / 4 + kRoundBlock - 1) / kRoundBlock);
  hipLaunchKernelGGL(host_round_kernel, dim3(grid), dim3(kRoundBlock), 0, st, rows, L, int(K), iw, res_d,
                     cx.counter, flag_d, seq);
  if (int rc = check_launch("fedagg_host_round_f32")) return rc;
  // the completion word; a bounded spin, then the stream's own error
  const auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(cx.flag, __ATOMIC_ACQUIRE) != seq) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      const hipError_t e = hipStreamSynchronize(st);
      if (e != hipSuccess) return set_error(static_cast<int>(e), "fedagg_host_round_f32: " + std::string(hipGetErrorString(e)));
      if (__atomic_load_n(cx.flag, __ATOMIC_ACQUIRE) != seq)
        return set_error(FEDAGG_EINVAL, "fedagg_host_round_f32: completion word never arrived");
      break;
    }
  }
  // unpack into the caller's per-key host tensors (fp32 results)
  split_rows(L * 4, T, [&](int t) {
    if (numels[t]) memcpy(h_out[t], cx.res + off[t], size_t(numels[t]) * 4);
  });
  return FEDAGG_OK;
}

const char* fedagg_last_error(void) { return g_last_error.c_str(); }

// error reporting for the other translation unit (csrc/robust.hip); not in
// the header, not exported from the library
__attribute__((visibility("hidden"))) int fedagg_set_error_internal(int code, const char* msg) {
  return set_error(code, msg);
}

int32_t fedagg_version(void) { return 1; }

#ifdef FEDAGG_TUNING  // the tuning entries (tools/tuning_lib.py)
int fedagg_wsum_f32_variant(const float* const* d_src, const float* d_w, int32_t K, int64_t N, float* d_out,
                            int32_t variant, fedagg_stream_t stream) {
  if (variant < 0 || variant >= kNumVariants) return set_error(FEDAGG_EINVAL, "bad variant");
  if (K < 1 || N < 0 || !d_src || !d_w || !d_out) return set_error(FEDAGG_EINVAL, "bad argument");
  if (N == 0) return FEDAGG_OK;
  return kVariants[variant].fn(d_src, d_w, K, N, d_out, reinterpret_cast<hipStream_t>(stream));
}

const char* fedagg_variant_name(int32_t variant) {
  if (variant < 0 || variant >= kNumVariants) return "";
  return kVariants[variant].name;
}

int32_t fedagg_num_variants(void) { return kNumVariants; }

int fedagg_wsum_tiny_variant(int32_t dtype, const void* const* d_src, const float* d_w, int32_t K, int64_t N,
                             void* d_out, int32_t variant, fedagg_stream_t stream) {
  if (variant < 0 || variant >= kNumTinyVariants) return set_error(FEDAGG_EINVAL, "bad variant");
  if (dtype != FEDAGG_DT_F32 && dtype != FEDAGG_DT_BF16 && dtype != FEDAGG_TUNE_BF16_F32OUT &&
      dtype != FEDAGG_TUNE_BF16_ACC32)
    return set_error(FEDAGG_EINVAL, "tiny variants: f32, bf16, bf16 -> f32 partial or bf16 fp32-accumulated");
  if (K < 1 || N < 0 || !d_src || !d_w || !d_out) return set_error(FEDAGG_EINVAL, "bad argument");
  const TinyVariant& v = kTinyVariants[variant];
  const TinyFn f = dtype == FEDAGG_DT_F32    ? v.f32
                   : dtype == FEDAGG_DT_BF16 ? v.bf16
                   : dtype == FEDAGG_TUNE_BF16_F32OUT ? v.bf16f32
                                                      : v.bf16acc32;
  if (!f) return set_error(FEDAGG_EINVAL, "variant not built for this dtype");
  if (N == 0) return FEDAGG_OK;
  return f(d_src, d_w, K, N, d_out, reinterpret_cast<hipStream_t>(stream));
}

const char* fedagg_tiny_variant_name(int32_t variant) {
  if (variant < 0 || variant >= kNumTinyVariants) return "";
  return kTinyVariants[variant].name;
}

int32_t fedagg_num_tiny_variants(void) { return kNumTinyVariants; }
#endif  // FEDAGG_TUNING

}  // extern "C"
