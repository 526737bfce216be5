/*
 * fedagg.h — C ABI of libfedagg.so, the MI355X (gfx950) server-side federated
 * aggregation kernels.
 *
 * This is the drop-in boundary for FedML's server-side FedAvg reduction.  Every
 * entry point below replaces one arithmetic loop of the reference:
 *
 *   FedMLAggOperator.agg -> model_aggregator -> torch_aggregator
 *     python/fedml/ml/aggregator/agg_operator.py:10-30, :223-234, :33-134
 *
 * Conventions (all entry points):
 *   - Every pointer argument is a DEVICE pointer; the caller allocates and owns
 *     it.  No entry point allocates, frees or synchronises: they are
 *     asynchronous, stream-ordered and capturable into a hipGraph.
 *   - A "source table" `d_src` is a device array of K device pointers, one per
 *     client, in the client order of the reference's raw_grad_list.
 *   - `d_w` holds the per-client weights precomputed on the host exactly as the
 *     reference does: w_i = float32(float64(n_i) / float64(sum_j n_j))
 *     (agg_operator.py:24-28 and :39; the Python float is rounded to the tensor
 *     opmath type float32 by torch's mul-by-scalar).
 *   - `flags` bit FEDAGG_ALIGNED16 asserts that every source and output pointer
 *     is 16-byte aligned; then the 16-byte vector path is used, otherwise a
 *     scalar path of identical arithmetic.
 *   - Return value: 0 on success, otherwise a FEDAGG_E* code or a hipError_t
 *     (> 0).  fedagg_last_error() returns a thread-local description.
 *   - Thread-safe: no mutable global state apart from the thread-local error.
 *
 * Arithmetic contract (bit-exact with the reference on the same inputs):
 *   acc = fl(p_0 * w_0);  acc = fl(acc + fl(p_i * w_i)) for i = 1..K-1,
 *   two separately rounded IEEE operations (never an FMA), clients in order.
 */
#ifndef FEDAGG_H_
#define FEDAGG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* hipStream_t is an opaque pointer; declared here so that callers (ctypes, cgo)
 * need no HIP headers.  Pass 0 for the null stream. */
typedef void* fedagg_stream_t;

#define FEDAGG_OK 0
#define FEDAGG_EINVAL (-1)      /* bad argument (K < 1, N < 0, null pointer) */
#define FEDAGG_ENOKERNEL (-2)   /* no kernel for this configuration */

#define FEDAGG_ALIGNED16 1u     /* flags: all pointers 16-byte aligned */
#define FEDAGG_HOST_WEIGHTS 2u  /* flags: d_w is a HOST array of K <= 256 weights,
                                   passed by value in the kernel arguments (no
                                   upload; the one exception to "device pointers") */

/* bf16 / f16 accumulation modes (see fedagg_wsum_bf16) */
#define FEDAGG_ACC_REFERENCE 0  /* round to bf16/f16 after every mul and add, as torch CPU does */
#define FEDAGG_ACC_FP32 1       /* accumulate in fp32, round once at the end */

/* ---- FedAvg / FedProx weighted sum ------------------------------------- */

/* fp32 clients -> fp32 average.
 * Replaces agg_operator.py:35-44 (FedAvg) and :45-54 (FedProx) for fp32 keys;
 * same arithmetic as simulation/sp/fedavg/fedavg_api.py:144-159 and
 * simulation/mpi/fedopt/FedOptAggregator.py:93-101.
 * Also used as the client-axis partial of the multi-GPU mode (w_i are then the
 * GLOBAL weights, the partial is over this GPU's clients only). */
int fedagg_wsum_f32(const float* const* d_src, const float* d_w, int32_t K,
                    int64_t N, float* d_out, uint32_t flags,
                    fedagg_stream_t stream);

/* bf16 clients -> bf16 average (agg_operator.py:35-44 for bf16 keys).
 * acc_mode FEDAGG_ACC_REFERENCE reproduces torch's CPU chain bit-exactly:
 *   acc = bf16(f32(p_0) * w_0);  acc = bf16(f32(acc) + f32(bf16(f32(p_i) * w_i))).
 * acc_mode FEDAGG_ACC_FP32 keeps an fp32 accumulator and rounds once. */
int fedagg_wsum_bf16(const uint16_t* const* d_src, const float* d_w, int32_t K,
                     int64_t N, uint16_t* d_out, int32_t acc_mode,
                     uint32_t flags, fedagg_stream_t stream);

/* bf16 clients -> fp32 partial (fp32 accumulate, no final rounding): the
 * per-GPU pre-reduction of the client-axis multi-GPU mode. */
int fedagg_wsum_bf16_f32out(const uint16_t* const* d_src, const float* d_w,
                            int32_t K, int64_t N, float* d_out,
                            uint32_t flags, fedagg_stream_t stream);

/* Round an fp32 vector to bf16 or f16 (RNE; NaN -> torch's canonical NaN for
 * bf16): the final step of the client-axis multi-GPU mode for 16-bit models,
 * whose per-GPU partials and reduce-scatter are fp32.  dtype is
 * FEDAGG_DT_BF16 or FEDAGG_DT_F16 (defined below). */
int fedagg_round_f32(int32_t dtype, const float* d_in, int64_t N, void* d_out,
                     fedagg_stream_t stream);

/* fp16 clients -> fp16 average; acc_mode as for bf16. */
int fedagg_wsum_f16(const uint16_t* const* d_src, const float* d_w, int32_t K,
                    int64_t N, uint16_t* d_out, int32_t acc_mode,
                    uint32_t flags, fedagg_stream_t stream);

/* fp64 clients -> fp64 average; d_w64 holds the float64 weights n_i / sum n
 * (a Python float times a double tensor is a double multiply). */
int fedagg_wsum_f64(const double* const* d_src, const double* d_w64, int32_t K,
                    int64_t N, double* d_out, uint32_t flags,
                    fedagg_stream_t stream);

/* int64 clients -> fp32 average.  torch promotes int64 * Python float to the
 * default dtype float32: acc = fl32(fl32(v_0) * w_0); acc = fl32(acc + fl32(fl32(v_i) * w_i)).
 * This is what happens to BatchNorm num_batches_tracked in the reference. */
int fedagg_wsum_i64_f32(const int64_t* const* d_src, const float* d_w,
                        int32_t K, int64_t N, float* d_out, uint32_t flags,
                        fedagg_stream_t stream);

/* ---- FedAvg_seq / FedDyn unweighted sum -------------------------------- */

/* out = p_0 + p_1 + ... + p_{K-1} in the source dtype, sequential order.
 * Replaces agg_operator.py:55-63 (FedAvg_seq) and :68-77 (FedDyn).  The
 * reference aliases client 0's tensor and adds into it in place; pass
 * d_out == d_src[0] (host-side value) to reproduce that.  dtype codes:
 * FEDAGG_DT_* below. */
#define FEDAGG_DT_F32 0
#define FEDAGG_DT_BF16 1
#define FEDAGG_DT_F16 2
#define FEDAGG_DT_F64 3
#define FEDAGG_DT_I64 4
#define FEDAGG_DT_I32 5
int fedagg_sum(int32_t dtype, const void* const* d_src, int32_t K, int64_t N,
               void* d_out, uint32_t flags, fedagg_stream_t stream);

/* ---- Multi-tensor (one launch over every state-dict key) --------------- */

/* T tensors ("keys") of one dtype, each with its own K client pointers and
 * element count, reduced in ONE launch (the per-key loop of agg_operator.py:36
 * becomes a segment table).  d_src is a [T][K] device pointer table, d_out a
 * [T] device pointer table, d_numel a [T] device int64 array, and
 * d_block_begin a [T+1] device int64 prefix array of workgroup offsets that the
 * host computed with fedagg_multi_blocks() for the same dtype and numels.
 * fedagg_wsum_multi takes FEDAGG_DT_F32, _BF16, _F16 (acc_mode as for
 * fedagg_wsum_bf16; outputs keep the dtype) or _I64 (float32 outputs). */
int64_t fedagg_multi_blocks(int32_t dtype, int64_t numel);
int fedagg_wsum_multi(int32_t dtype, int32_t acc_mode, const void* const* d_src,
                      void* const* d_out, const int64_t* d_numel,
                      const int64_t* d_block_begin, int32_t T, const float* d_w,
                      int32_t K, int64_t total_blocks, fedagg_stream_t stream);
int fedagg_wsum_multi_f32(const float* const* d_src, float* const* d_out,
                          const int64_t* d_numel, const int64_t* d_block_begin,
                          int32_t T, const float* d_w, int32_t K,
                          int64_t total_blocks, fedagg_stream_t stream);

/* ---- MPI simulation FedAvg order --------------------------------------- */

/* out = sum_i fl( fl(p_i * n_i) / N ) in client order: the term order of the
 * MPI simulation's FedAVGAggregator._fedavg_aggregation_
 * (simulation/mpi/fedavg/FedAVGAggregator.py:99-116, `local_model_params[k] *
 * local_sample_number / training_num`), two roundings per client where the
 * plugin path (fedagg_wsum_*) has fl(p * fl(n_i / N)).  d_w is a DEVICE array
 * of K weight records of the dtype's layout:
 *   FEDAGG_DT_F32 / _BF16 / _F16: {float n, float d}    (fl32(n_i), fl32(N))
 *   FEDAGG_DT_F64:                {double n, double d}
 *   FEDAGG_DT_I64:                {int64 n, float nf, float d, int32 is_int, int32 pad}
 *     (is_int: n_i is an integer and multiplies in int64 with wrap-around;
 *      else fl32(v) * nf; the result is float32, as torch's true division)
 * bf16 / f16 round after the mul, the div and the add (torch's CPU chain).
 * Outputs keep the dtype (float32 for int64).  FEDAGG_HOST_WEIGHTS is refused. */
int fedagg_wsum_muldiv(int32_t dtype, const void* const* d_src, const void* d_w,
                       int32_t K, int64_t N, void* d_out, uint32_t flags,
                       fedagg_stream_t stream);

/* ---- FedOpt server step (fused epilogue) ------------------------------- */

/* Server SGD with momentum over named parameters, fused with the pseudo
 * gradient (simulation/mpi/fedopt/FedOptAggregator.py:104-130 with
 * torch.optim.SGD, dampening 0, nesterov False, weight_decay 0):
 *   g     = p_old - p_avg
 *   buf   = first_step ? g : fl(fl(buf * momentum) + g)
 *   p_new = p_old - lr * buf          (fused multiply-add, as torch's
 *                                      vectorised add_(buf, alpha=-lr))
 * d_param is updated in place, d_mom too (momentum == 0 leaves it unused). */
int fedagg_fedopt_sgd_f32(float* d_param, float* d_mom, const float* d_avg,
                          int64_t N, float lr, float momentum,
                          int32_t first_step, fedagg_stream_t stream);

/* FedAvg of K fp32 clients fused with the server SGD step above, in ONE pass:
 * the average is formed in registers and never written to HBM (saves 2·N·4 B
 * against fedagg_wsum_f32 + fedagg_fedopt_sgd_f32).  Bit-identical to that
 * two-kernel sequence and to FedOptAggregator.aggregate's named-parameter
 * update (FedOptAggregator.py:93-112, :118-125).  d_param holds p_old on entry
 * and p_new on return; d_mom the momentum buffer (unused if momentum == 0). */
int fedagg_wsum_fedopt_sgd_f32(const float* const* d_src, const float* d_w,
                               int32_t K, int64_t N, float* d_param,
                               float* d_mom, float lr, float momentum,
                               int32_t first_step, uint32_t flags,
                               fedagg_stream_t stream);

/* Server Adam (torch.optim.Adam defaults: amsgrad off, weight_decay 0) fused
 * with the FedAvg of K fp32 clients, one pass.  Replaces the server step of
 * simulation/sp/fedopt/fedopt_api.py:121-130 (_set_model_global_grads, then
 * opt.step() with OptRepo "adam", lr=server_lr).  d_exp_avg / d_exp_avg_sq are
 * the optimizer state (N floats each, zero before the first step; with
 * first_step != 0 they are only written).  scalars6 is host memory filled by
 * fedagg_adam_scalars() for the step number (1-based) about to be taken.
 * Per element: g = p - avg; m = lerp(m, g, 1-beta1); v = v*beta2 + (1-beta2)*g*g;
 * p += (-lr/bc1)*m / (sqrt(v)/sqrt(bc2) + eps), rounded as torch's CPU kernels
 * round (lerp and addcmul fused, addcdiv not); sqrt is correctly rounded. */
int fedagg_adam_scalars(double lr, double beta1, double beta2, double eps,
                        int64_t step, float* out6);
int fedagg_wsum_fedopt_adam_f32(const float* const* d_src, const float* d_w,
                                int32_t K, int64_t N, float* d_param,
                                float* d_exp_avg, float* d_exp_avg_sq,
                                const float* scalars6, int32_t first_step,
                                uint32_t flags, fedagg_stream_t stream);

/* Server Adagrad (torch.optim.Adagrad: weight_decay 0) fused with the FedAvg
 * of K fp32 clients, one pass.  Replaces the server step of
 * simulation/sp/fedopt/fedopt_api.py:121-130 with OptRepo "adagrad"
 * (optrepo.py:10-38 builds torch.optim.Adagrad(params, lr=server_lr)).
 * d_sum is the optimizer's state_sum (N floats; initial_accumulator_value,
 * i.e. zeros, before the first step).  clr = lr / (1 + (step-1) * lr_decay),
 * the step's learning rate as torch computes it in double (= lr for FedML).
 * Per element: g = p - avg; sum = fma(g, g, sum);
 * p = p + fl(-clr * g) / (sqrt(sum) + eps), rounded as torch's CPU kernels
 * round (addcmul fused, addcdiv not); sqrt is correctly rounded. */
int fedagg_wsum_fedopt_adagrad_f32(const float* const* d_src, const float* d_w,
                                   int32_t K, int64_t N, float* d_param,
                                   float* d_sum, float clr, float eps,
                                   uint32_t flags, fedagg_stream_t stream);

/* FedAvg fused with the server AdamW step (torch.optim.AdamW through
 * OptRepo "adamw", sp/fedopt/optrepo.py:10-38, as FedOptAPI builds it with
 * lr only, fedopt_api.py:78-85): Adam as fedagg_wsum_fedopt_adam_f32 on the
 * gradient p_old - avg, with the parameter first scaled by
 * decay = fl32(1 - lr * weight_decay) (decoupled weight decay):
 *   p = fl(p_old * decay) + fl(-step_size * m) / denom. */
int fedagg_wsum_fedopt_adamw_f32(const float* const* d_src, const float* d_w,
                                 int32_t K, int64_t N, float* d_param,
                                 float* d_exp_avg, float* d_exp_avg_sq,
                                 const float* scalars6, float decay,
                                 int32_t first_step, uint32_t flags,
                                 fedagg_stream_t stream);

/* FedAvg fused with the server RMSprop step (torch.optim.RMSprop, OptRepo
 * "rmsprop", defaults momentum 0, centered False, weight_decay 0):
 *   g = p_old - avg
 *   square_avg = fma(fl(fl32(1 - alpha) * g), g, fl(square_avg * fl32(alpha)))
 *   p = p_old + fl(fl(-lr * g) / fl(sqrt(square_avg) + eps))
 * alpha is the Python float (double); square_avg starts at zero. */
int fedagg_wsum_fedopt_rmsprop_f32(const float* const* d_src, const float* d_w,
                                   int32_t K, int64_t N, float* d_param,
                                   float* d_square_avg, float lr, double alpha,
                                   float eps, uint32_t flags,
                                   fedagg_stream_t stream);

/* The other elementwise optimizers OptRepo names (sp/fedopt/optrepo.py:10,
 * torch.optim's direct Optimizer subclasses), each as FedOptAPI builds it
 * with lr only (fedopt_api.py:78-85) and steps it (:121-130), fused with the
 * FedAvg of K fp32 clients in one pass.  opt selects the optimizer; state0 /
 * state1 are its per-element buffers in the state torch creates before its
 * first step:
 *   FEDAGG_OPT_ADAMAX    exp_avg / exp_inf       (zeros)
 *   FEDAGG_OPT_NADAM     exp_avg / exp_avg_sq    (zeros)
 *   FEDAGG_OPT_RADAM     exp_avg / exp_avg_sq    (zeros)
 *   FEDAGG_OPT_ADADELTA  square_avg / acc_delta  (zeros)
 *   FEDAGG_OPT_ASGD      ax / unused (may be NULL)  (zeros)
 *   FEDAGG_OPT_RPROP     prev / step_size        (zeros / fl32(lr))
 * scalars9 (host memory) comes from fedagg_optrepo_scalars() for the 1-based
 * step about to be taken; carry2 is the optimizer's fp32 scalar state, updated
 * by that call: NAdam's mu_product (1.0 before the first step), ASGD's eta and
 * mu (fl32(lr), 1.0), ignored otherwise.  Per element each step rounds as
 * torch 2.10's single-tensor CPU path (lerp_ / addcmul_ / add_(alpha) fused,
 * addcdiv_ not; the formulas beside OptRepoEpi in csrc/fedagg.hip); sqrt is
 * correctly rounded, so NAdam / RAdam / Adadelta differ from torch's MKL sqrt
 * by its rounding only (Adamax, ASGD and Rprop take no sqrt: bit-exact). */
#define FEDAGG_OPT_ADAMAX 1
#define FEDAGG_OPT_NADAM 2
#define FEDAGG_OPT_RADAM 3
#define FEDAGG_OPT_ADADELTA 4
#define FEDAGG_OPT_ASGD 5
#define FEDAGG_OPT_RPROP 6
int fedagg_optrepo_scalars(int32_t opt, double lr, int64_t step, float* carry2,
                           float* out9);
int fedagg_wsum_fedopt_optrepo_f32(int32_t opt, const float* const* d_src,
                                   const float* d_w, int32_t K, int64_t N,
                                   float* d_param, float* d_state0,
                                   float* d_state1, const float* scalars9,
                                   uint32_t flags, fedagg_stream_t stream);

/* Every fused server launch of one FedOpt round in ONE call: the launches of
 * a server process that drives several GPUs (MultiDeviceFedOptServer: each
 * GPU its keys, FedOptAggregator.py:81-130 over the whole model), issued in
 * order, each on its own device and stream (the calling thread's current
 * device is restored).  A launch is the entry point its `opt` names, with the
 * descriptor's fields as that entry's arguments:
 *   FEDAGG_FEDOPT_AVG      the plain FedAvg of `dtype` rows into d_param:
 *                          fedagg_wsum_f32 / _bf16 / _f16 (acc_mode) / _f64 (double
 *                          weights) / _i64_f32 (buffer keys of a FedOpt round, and
 *                          every device's reduction of a one-process multi-GPU round)
 *   FEDAGG_FEDOPT_SGD      fedagg_wsum_fedopt_sgd_f32 (d_state0 = momentum)
 *   FEDAGG_FEDOPT_ADAM     fedagg_wsum_fedopt_adam_f32 (scalars = adam scalars6)
 *   FEDAGG_FEDOPT_ADAMW    fedagg_wsum_fedopt_adamw_f32 (+ decay)
 *   FEDAGG_FEDOPT_ADAGRAD  fedagg_wsum_fedopt_adagrad_f32 (lr = clr)
 *   FEDAGG_FEDOPT_RMSPROP  fedagg_wsum_fedopt_rmsprop_f32 (+ alpha)
 *   FEDAGG_OPT_*           fedagg_wsum_fedopt_optrepo_f32 (scalars = scalars9)
 * Stops at the first failing launch and returns its code. */
#define FEDAGG_FEDOPT_AVG 0
#define FEDAGG_FEDOPT_SGD 16
#define FEDAGG_FEDOPT_ADAM 17
#define FEDAGG_FEDOPT_ADAMW 18
#define FEDAGG_FEDOPT_ADAGRAD 19
#define FEDAGG_FEDOPT_RMSPROP 20
typedef struct fedagg_fedopt_launch {
  const float* const* d_src;  /* device table of K client pointers */
  const float* weights;       /* device array, or host with FEDAGG_HOST_WEIGHTS */
  float* d_param;
  float* d_state0;
  float* d_state1;
  const float* scalars;       /* host */
  fedagg_stream_t stream;
  int64_t N;
  double alpha;
  float lr, momentum, eps, decay;
  int32_t K, opt, device, first_step;
  uint32_t flags;
  int32_t dtype;              /* FEDAGG_FEDOPT_AVG: FEDAGG_DT_* of the rows (0 = fp32) */
  int32_t acc_mode;           /* FEDAGG_FEDOPT_AVG of bf16 / f16 rows */
  int32_t reserved;
} fedagg_fedopt_launch;
int fedagg_wsum_fedopt_batch(const fedagg_fedopt_launch* launches, int32_t n);

/* ---- Robust aggregation --------------------------------------------------- */

/* Coordinate-wise median over K fp32 clients (the "wise_median" defense,
 * core/security/defense/coordinate_wise_median_defense.py:24-32:
 * torch.median(stack, dim=-1).values): out[e] = the LOWER median (sorted
 * element (K-1)/2) of {src_i[e]}; if the column holds a NaN, the first NaN in
 * client order.  Any K >= 1 and N (K <= 128: one lane per element, a pruned
 * sorting network in registers, launched in chunks of 2^30 columns;
 * 128 < K <= 4096: 4 to 32 lanes per element, each sorting 64 or 128
 * values in registers, merged across lanes; otherwise an 8-bit MSD radix
 * select per column over LDS histograms, the column re-read per digit).  Where +0.0 and
 * -0.0 tie at the median the sign of the zero returned may differ from
 * torch's (nth_element order). */
int fedagg_median_f32(const float* const* d_src, int32_t K, int64_t N,
                      float* d_out, uint32_t flags, fedagg_stream_t stream);

/* The same median for dtype FEDAGG_DT_F32, _BF16 or _F16 rows (d_src and
 * d_out of that dtype): a bf16 / f16 model's stack, torch.median over it
 * (torch.cat keeps the 16-bit dtype).  Values are widened to fp32 exactly,
 * selected, and the selected input narrowed back exactly; a NaN column
 * returns a NaN.  With FEDAGG_ALIGNED16 (16-byte aligned rows and output)
 * 16-bit rows up to K = 4096 take the packed kernels instead: up to 128
 * clients two columns per register as order-preserving int16 keys on the same
 * networks (v_pk_min_i16 / v_pk_max_i16); 129 to 1024 clients a radix select
 * on bit planes of the order keys, the rows streamed through LDS by LDS-DMA;
 * above that sorting networks over lane groups. */
int fedagg_median(int32_t dtype, const void* const* d_src, int32_t K,
                  int64_t N, void* d_out, uint32_t flags,
                  fedagg_stream_t stream);

/* Distance-based defenses (csrc/robust.hip).  Rows are K fp32 device
 * pointers; the columns that count (FedML's vectorize_weight: every key but
 * BatchNorm running stats and counters, core/security/common/utils.py:8-21)
 * arrive as d_chunks, n_chunks (start, length) int64 pairs of row columns,
 * each length <= the kernel's chunk size (FEDAGG_DIST_CHUNK for dist2,
 * FEDAGG_PAIR_CHUNK for pairdist2).  Differences are the reference's fp32
 * differences.  dist2 squares and sums them in fp64; pairdist2 squares and
 * sums them in fp32 over stages of <= 64 columns and adds the stage sums in
 * fp64 (relative error ~1e-7, the reference's own fp32 norm's order).
 * Per-block partials sit in d_work and are combined in a fixed order: the
 * results are deterministic.  d_work holds at least
 * fedagg_robust_work_len(kind, K, n_chunks) doubles.
 *
 * fedagg_dist2_f32 replaces the per-client torch.norm(vec_local - vec_global)
 * of NormDiffClippingDefense._get_clipped_norm_diff
 * (defense/norm_diff_clipping_defense.py:38-42) and CClip's
 * compute_euclidean_distance (cclip_defense.py:72-80):
 *   d_out[i] = sum_e (src_i[e] - ref[e])^2   (fp64; ref NULL: plain norms).
 *
 * fedagg_pairdist2_f32 replaces KrumDefense._compute_krum_score's K(K-1)
 * compute_euclidean_distance(v_i, v_j) (defense/krum_defense.py:47-60):
 *   d_out[i*K + j] = sum_e (src_i[e] - src_j[e])^2   (fp64, symmetric, 0 on
 *   the diagonal). */
#define FEDAGG_DIST_CHUNK 1024
#define FEDAGG_PAIR_CHUNK 256
#define FEDAGG_WORK_DIST2 0
#define FEDAGG_WORK_PAIRDIST2 1
#define FEDAGG_WORK_PAIRGRAM 2
int64_t fedagg_robust_work_len(int32_t kind, int32_t K, int64_t n_chunks);
int fedagg_dist2_f32(const float* const* d_src, int32_t K, const float* d_ref,
                     const int64_t* d_chunks, int64_t n_chunks, double* d_out,
                     double* d_work, int64_t work_len, fedagg_stream_t stream);
int fedagg_pairdist2_f32(const float* const* d_src, int32_t K,
                         const int64_t* d_chunks, int64_t n_chunks, double* d_out,
                         double* d_work, int64_t work_len, fedagg_stream_t stream);

/* The same K x K matrix as fedagg_pairdist2_f32 (the same replaced lines,
 * krum_defense.py:47-60) for K <= 128, as a centred Gram on the bf16 matrix
 * cores: per 64-column stage c = x - (column mean over the K clients), each
 * c split exactly into three bf16 parts h + m + l, G = C C^T from six
 * v_mfma_f32_16x16x32_bf16 products per 32 columns (hh, hm, mh, mm, hl, lh;
 * fp32 over 4 stages, fp64 across), d_out[i*K + j] = max(0, G_ii + G_jj -
 * (G_ij + G_ji)).  Not the reference's fp32 differences: |error| ~ 1e-7
 * (|c_i|^2 + |c_j|^2), the order of the reference's own fp32 torch.norm when
 * the clients are spread about as far as they are apart.  d_work: fedagg_robust_work_len(FEDAGG_WORK_PAIRGRAM,
 * K, n_chunks) doubles (-1 there for K > 128). */
int fedagg_pairgram2_f32(const float* const* d_src, int32_t K,
                         const int64_t* d_chunks, int64_t n_chunks, double* d_out,
                         double* d_work, int64_t work_len, fedagg_stream_t stream);

/* The clipped rebuild of NormDiffClippingDefense (:38-54): over the first N
 * columns of every row,
 *   d_dst_i[e] = fl32( fl32( fl32(src_i[e] - ref[e]) / d_div[i] ) + ref[e] )
 * with d_div[i] = fl32(max(1, norm_i / norm_bound)), the Python divisor torch
 * applies to the fp32 difference vector (K device floats). */
int fedagg_clip_diff_f32(const float* const* d_src, int32_t K, const float* d_ref,
                         const float* d_div, int64_t N, float* const* d_dst,
                         fedagg_stream_t stream);

/* CClip's scaled differences (CClipDefense.defend_before_aggregation,
 * defense/cclip_defense.py:47-52, over every key of the bucket means):
 *   d_dst_i[e] = fl32( fl32(src_i[e] - ref[e]) * d_scale[i] )
 * with d_scale[i] = fl32(min(1, tau / (norm_i + 1e-8))) (K device floats). */
int fedagg_scale_diff_f32(const float* const* d_src, int32_t K, const float* d_ref,
                          const float* d_scale, int64_t N, float* const* d_dst,
                          fedagg_stream_t stream);

/* The robust-learning-rate defense (RobustLearningRateDefense.run,
 * core/security/defense/robust_learning_rate_defense.py:35-62, reached through
 * FedMLDefender.defend from simulation/mpi/fedavg/FedAVGAggregator.py:83-88):
 * per element, the FedAvg chain of fedagg_wsum_f32 (avg) and the sum of the
 * clients' torch.sign values (s), in one pass; then
 *   lr = |s|; lr = lr < thr ? -1 : lr; lr = lr >= thr ? 1 : lr; out = lr * avg
 * (a NaN input leaves lr, and so out, NaN).  threshold = fl32 of the config's
 * robust_threshold (!= 0; 0 means plain aggregation, handled by the caller).
 * Flags as fedagg_wsum_f32. */
int fedagg_wsum_rlr_f32(const float* const* d_src, const float* d_w, int32_t K,
                        int64_t N, float threshold, float* d_out, uint32_t flags,
                        fedagg_stream_t stream);

/* Secure aggregation in a finite field (LightSecAgg), numpy int64 semantics:
 * wrapping adds, floor modulo.  p > 0.
 *
 * fedagg_sum_mod_i64 replaces aggregate_models_in_finite
 * (core/mpc/lightsecagg.py:134-148): out = x_0; out = (out + x_i) mod p.
 *
 * fedagg_lsa_reconstruct_f32 replaces the per-key loop of
 * LightSecAggAggregator.aggregate_model_reconstruction
 * (cross_silo/lightsecagg/lsa_fedml_aggregator.py:139-166) with
 * transform_finite_to_tensor / my_q_inv (lightsecagg.py:157-182):
 *   m = (Σ_i x_i − mask) mod p;  v = m > (p−1)/2 ? m − p : m  (float64);
 *   out = fl32( fl32(v / 2^q_bits) · w )   with w = fl32(1 / K_active).
 * d_mask is the decoded aggregate mask laid out like the client rows. */
int fedagg_sum_mod_i64(const int64_t* const* d_src, int32_t K, int64_t N,
                       int64_t p, int64_t* d_out, uint32_t flags,
                       fedagg_stream_t stream);
int fedagg_lsa_reconstruct_f32(const int64_t* const* d_src, int32_t K, int64_t N,
                               const int64_t* d_mask, int64_t p, int32_t q_bits,
                               float w, float* d_out, uint32_t flags,
                               fedagg_stream_t stream);

/* ---- Host ingest helper -------------------------------------------------- */

/* HOST-side gather of n host buffers into one host buffer (normally pinned
 * staging for a single H2D per client): srcs[i] (nbytes[i] bytes) goes to
 * dst + dst_offs[i].  The total is split into `threads` contiguous byte
 * ranges copied in parallel.  This is the packing step of the ingest path that
 * replaces the reference's per-key tensor.to(device) at client arrival
 * (ml_engine_adapter.py:234-254).  Synchronous; touches no device memory. */
int fedagg_host_pack(void* dst, const void* const* srcs, const int64_t* dst_offs,
                     const int64_t* nbytes, int32_t n, int32_t threads);

/* The inverse scatter for the broadcast side: src + src_offs[i] goes to
 * dsts[i] (one host tensor per state-dict key, as the reference returns). */
int fedagg_host_unpack(const void* src, void* const* dsts, const int64_t* src_offs,
                       const int64_t* nbytes, int32_t n, int32_t threads);

/* The general form for a client spread over several destinations: srcs[i]
 * (nbytes[i] bytes) goes to dsts[i].  A round cut over G GPUs (whole keys per
 * GPU, fedml_amd.multidev) packs every GPU's pinned staging row of an arriving
 * client in ONE call, so the G per-GPU H2Ds can be issued together right
 * after it (the packing half of add_local_trained_result's tensor moves,
 * cross_silo/server/fedml_aggregator.py:58-67).  Synchronous; host memory only. */
int fedagg_host_gather(void* const* dsts, const void* const* srcs, const int64_t* nbytes, int32_t n,
                       int32_t threads);

/* ---- Small device-resident rounds --------------------------------------- */

/* One whole FedAvg round of DEVICE tensors in one launch: the reference call
 * shape FedMLAggOperator.agg(args, [(n_i, gpu_state_dict)]) (agg_operator.py:
 * 35-44, the server's `using_gpu` mode, ml_engine_adapter.py:234-254) for
 * rounds of at most 16 keys and 128 client tensors (config 1: 4 clients x 2
 * keys), where uploads and launches, not bytes, are the cost.
 *   d_src   : host array of device pointers [T][K], key-major (key t of
 *             client i at t*K + i), 16-byte aligned
 *   codes   : FEDAGG_DT_F32 or FEDAGG_DT_I64 per key (int64 values enter as
 *             fl32(v) and give fp32 results, the reference's promotion)
 *   weights : K fp32 weights fl32(n_i / sum n), host memory
 *   d_out   : host array of T device fp32 buffers (16-byte aligned)
 * Every pointer, length and weight travels in the kernel arguments (no
 * upload, no allocation); asynchronous and ordered on `stream`.
 * Bit-identical to the reference chain. */
int fedagg_device_round_f32(const void* const* d_src, const int32_t* codes,
                            const int64_t* numels, int32_t T, int32_t K,
                            const float* weights, void* const* d_out,
                            fedagg_stream_t stream);

/* ---- Small host-resident rounds ----------------------------------------- */

/* One whole FedAvg round of HOST tensors, host to host, in one call: the
 * reference call shape FedMLAggOperator.agg(args, [(n_i, cpu_state_dict)])
 * (agg_operator.py:35-44; the SP simulation's FedAvgAPI._aggregate,
 * simulation/sp/fedavg/fedavg_api.py:144-159) for rounds small enough that a
 * PCIe round trip, not bytes, is the cost (configs 1 and 2).
 *   h_src   : host pointers [T][K], key-major: key t of client i at t*K + i
 *   codes   : FEDAGG_DT_F32 or FEDAGG_DT_I64 per key (int64 values enter as
 *             fl32(v) and give fp32 results, the reference's promotion)
 *   weights : K fp32 weights fl32(n_i / sum n), K <= 256
 *   h_out   : T host fp32 buffers of numels[t] elements, written on return
 * The library packs the clients into pinned memory it keeps per device
 * (allocated on first use and grown when a bigger round arrives), reduces on
 * the device (the kernel reads rounds up to 16 MiB straight from pinned
 * memory; larger ones go up in pipelined DMAs), and copies the result out.
 * Synchronous (returns when h_out holds the result).  stream NULL runs it
 * on a non-blocking stream of the library's own (nothing on the caller's
 * streams is involved: host in, host out); a stream orders it after the
 * caller's work there.  Bit-identical to the reference chain. */
int fedagg_host_round_f32(const void* const* h_src, const int32_t* codes,
                          const int64_t* numels, int32_t T, int32_t K,
                          const float* weights, void* const* h_out,
                          fedagg_stream_t stream);

/* ---- Introspection ------------------------------------------------------ */
const char* fedagg_last_error(void);
int32_t fedagg_version(void);


#ifdef __cplusplus
}
#endif

#endif /* FEDAGG_H_ */
