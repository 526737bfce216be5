/*
 * fedavg_oracle.c — CPU restatement of FedML's server-side aggregation
 * arithmetic.  TEST INFRASTRUCTURE ONLY: it is the checker for the HIP path
 * (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg).  The product
 * path (fedml_amd/) never links, loads or calls it.
 *
 * Reference: python/fedml/ml/aggregator/agg_operator.py
 *   FedAvg / FedProx   :35-54   avg[k] = p_0[k]*w_0 ; avg[k] += p_i[k]*w_i
 *   FedAvg_seq/FedDyn  :55-63, :68-77   avg[k] = p_0[k] ; avg[k] += p_i[k]
 * and the FedOpt server step of
 *   python/fedml/simulation/mpi/fedopt/FedOptAggregator.py:104-130
 *   (torch.optim.SGD, momentum, dampening 0).
 *
 * The arithmetic inside those Python lines is torch's CPU elementwise kernels;
 * their rounding is restated here per dtype (see each function).  Compile with
 * -ffp-contract=off so that `a + b * c` stays two roundings; the one fused
 * operation (SGD's add_(buf, alpha=-lr), a vectorised fmadd in torch) uses
 * fmaf() explicitly.
 *
 * Single-threaded scalar loops: simple enough to audit line by line.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* c10::BFloat16 round_to_nearest_even (NaN -> 0x7FC0). */
uint16_t oracle_f32_to_bf16(float f) {
  uint32_t u = f2u(f);
  if (isnan(f)) return 0x7fc0;
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
float oracle_bf16_to_f32(uint16_t h) { return u2f((uint32_t)h << 16); }
static float rbf(float f) { return oracle_bf16_to_f32(oracle_f32_to_bf16(f)); }

/* agg_operator.py:36-44 on fp32 keys.  `p * w` with w a Python float is
 * fl32(p * fl32(w)) (torch casts the scalar to the opmath type float);
 * `acc += t` is fl32(acc + t).  src is K row pointers of N floats. */
void oracle_wsum_f32(const float* const* src, const float* w, int K, int64_t N, float* out) {
  for (int64_t e = 0; e < N; ++e) {
    float acc = src[0][e] * w[0];
    for (int i = 1; i < K; ++i) {
      float t = src[i][e] * w[i];
      acc = acc + t;
    }
    out[e] = acc;
  }
}

/* Same lines on bf16 keys: opmath float, rounded to bf16 after the mul and
 * after the add (the product is materialised as a bf16 tensor, then add_). */
void oracle_wsum_bf16(const uint16_t* const* src, const float* w, int K, int64_t N, uint16_t* out) {
  for (int64_t e = 0; e < N; ++e) {
    float acc = rbf(oracle_bf16_to_f32(src[0][e]) * w[0]);
    for (int i = 1; i < K; ++i) {
      float t = rbf(oracle_bf16_to_f32(src[i][e]) * w[i]);
      acc = rbf(acc + t);
    }
    out[e] = oracle_f32_to_bf16(acc);
  }
}

/* int64 keys (e.g. BatchNorm num_batches_tracked): int64 * Python float
 * promotes to float32, computed as fl32(fl32(v) * fl32(w)). */
void oracle_wsum_i64_f32(const int64_t* const* src, const float* w, int K, int64_t N, float* out) {
  for (int64_t e = 0; e < N; ++e) {
    float acc = (float)src[0][e] * w[0];
    for (int i = 1; i < K; ++i) {
      float t = (float)src[i][e] * w[i];
      acc = acc + t;
    }
    out[e] = acc;
  }
}

/* fp64 keys: double * Python float is a double multiply. */
void oracle_wsum_f64(const double* const* src, const double* w, int K, int64_t N, double* out) {
  for (int64_t e = 0; e < N; ++e) {
    double acc = src[0][e] * w[0];
    for (int i = 1; i < K; ++i) {
      double t = src[i][e] * w[i];
      acc = acc + t;
    }
    out[e] = acc;
  }
}

/* agg_operator.py:55-63 (FedAvg_seq) on fp32 keys: plain sequential sum. */
void oracle_sum_f32(const float* const* src, int K, int64_t N, float* out) {
  for (int64_t e = 0; e < N; ++e) {
    float acc = src[0][e];
    for (int i = 1; i < K; ++i) acc = acc + src[i][e];
    out[e] = acc;
  }
}

/* FedAvg_seq on bf16 keys: bf16(f32(a) + f32(b)) per add_. */
void oracle_sum_bf16(const uint16_t* const* src, int K, int64_t N, uint16_t* out) {
  for (int64_t e = 0; e < N; ++e) {
    float acc = oracle_bf16_to_f32(src[0][e]);
    for (int i = 1; i < K; ++i) acc = rbf(acc + oracle_bf16_to_f32(src[i][e]));
    out[e] = oracle_f32_to_bf16(acc);
  }
}

/* FedAvg_seq on int64 keys: two's-complement wrapping adds. */
void oracle_sum_i64(const int64_t* const* src, int K, int64_t N, int64_t* out) {
  for (int64_t e = 0; e < N; ++e) {
    uint64_t acc = (uint64_t)src[0][e];
    for (int i = 1; i < K; ++i) acc += (uint64_t)src[i][e];
    out[e] = (int64_t)acc;
  }
}

/* FedOptAggregator.py:104-112,118-125 with torch.optim.SGD (momentum m,
 * dampening 0, no nesterov, no weight decay), one named parameter:
 *   grad = p_old - p_avg                          (:123, one rounding)
 *   buf  = first ? grad : fl(fl(buf * m) + grad)  (SGD: buf.mul_(m).add_(grad))
 *   p    = fma(buf, -lr, p_old)                   (SGD: p.add_(buf, alpha=-lr);
 *                                                  torch's CPU add is a fused
 *                                                  multiply-add)
 * With m == 0 torch skips the buffer and steps with grad directly. */
void oracle_fedopt_sgd_f32(float* p, float* buf, const float* avg, int64_t N, float lr, float m, int first) {
  const float neg_lr = -lr;
  for (int64_t e = 0; e < N; ++e) {
    const float po = p[e];
    const float g = po - avg[e];
    float b = g;
    if (m != 0.0f) {
      if (!first) {
        float t = buf[e] * m;
        b = t + g;
      }
      buf[e] = b;
    }
    p[e] = fmaf(b, neg_lr, po);
  }
}

/* torch.optim.Adam, single-tensor CPU path (torch/optim/adam.py
 * _single_tensor_adam), the moment updates of one step:
 *   g = p - avg                          fedopt_api.py:160 parameter.grad
 *   m.lerp_(g, w1)                       ATen lerp: |w1| < 0.5 ? fma(w1, g-m, m)
 *                                                   : fma(w1-1, g-m, g)
 *   v.mul_(beta2).addcmul_(g, g, c2)     fma(fl(c2*g), g, fl(v*beta2))
 * (fusion measured against torch 2.10's CPU kernels, vector body and scalar
 * tail).  The parameter update needs torch's own sqrt and is done by the
 * caller (fedavg_oracle.fedopt_adam). */
void oracle_adam_moments_f32(const float* p, const float* avg, float* m, float* v, int64_t N, float w1, float beta2,
                             float c2) {
  const int small = fabsf(w1) < 0.5f;
  for (int64_t e = 0; e < N; ++e) {
    const float g = p[e] - avg[e];
    const float d = g - m[e];
    m[e] = small ? fmaf(w1, d, m[e]) : fmaf(w1 - 1.0f, d, g);
    const float vb = v[e] * beta2;
    v[e] = fmaf(c2 * g, g, vb);
  }
}

/* Server Adagrad's accumulator (sp/fedopt/fedopt_api.py:121-130 with
 * torch.optim.Adagrad, single-tensor CPU path): g = p - avg;
 *   state_sum.addcmul_(g, g, value=1)    fma(g, g, sum)  (fl(1*g) = g)
 * (measured against torch 2.10's CPU kernel, vector body and scalar tail).
 * The parameter update needs torch's own sqrt and is done by the caller
 * (fedavg_oracle.fedopt_adagrad). */
void oracle_adagrad_sum_f32(const float* p, const float* avg, float* sum, int64_t N) {
  for (int64_t e = 0; e < N; ++e) {
    const float g = p[e] - avg[e];
    sum[e] = fmaf(g, g, sum[e]);
  }
}

/* out = fmaf(a, b, c) elementwise: the fused multiply-adds of torch's CPU
 * lerp_ / addcmul_ / add_(alpha) kernels, for the numpy restatements of the
 * server optimizers (fedavg_oracle.py fedopt_step). */
void oracle_fma_f32(const float* a, const float* b, const float* c, float* out, int64_t N) {
  for (int64_t e = 0; e < N; ++e) out[e] = fmaf(a[e], b[e], c[e]);
}
