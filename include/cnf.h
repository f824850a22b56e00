/*
 * cnf.h -- C ABI of libcnf_hip.so, the MI355X (gfx950) coupling-flow engine.
 *
 * Drop-in native boundary for the RealNVP / NICE forward, inverse and
 * log|det J| path of the reference (SergioAlvarezB/calibration-normalizing-flows):
 *
 *   cnf_forward   replaces Flow.forward            flows/flows.py:17-25
 *                 (NvpCouplingLayer.forward         flows/flows.py:101-112,
 *                  MLP.forward                      flows/utils.py:26-31)
 *   cnf_inverse   replaces Flow.backward           flows/flows.py:27-37
 *                 (NvpCouplingLayer.backward        flows/flows.py:114-126 -- the
 *                  reference's "backward" is the INVERSE transform, not autograd)
 *   cnf_prepare   replaces the per-layer parameter reads of the above
 *                 (state_dict layout: flows/flows.py:76-99, flows/utils.py:14-22)
 *   cnf_loss_vjp  replaces autograd of the calibrator loss
 *                 calibrators.py:287-295 / run_experiment3D.py:102-107
 *
 * Plain C: pointers + sizes, no torch types.  Every device pointer is a HIP
 * device allocation owned by the caller; all work is enqueued on the caller's
 * stream (hipStream_t passed as void*), nothing synchronises the host, nothing
 * allocates, so every entry point is graph-capturable (cnf_prepare included
 * once its host tables are built -- see below).  Errors are returned as
 * negative cnf_status codes; no exception crosses the ABI.
 *
 * Data layout: row-major fp32 logit batches [B][D] (one logit vector per row).
 */
#ifndef CNF_H_
#define CNF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CNF_ABI_VERSION 2   /* 2: cnf_adam_step takes double hyper-parameters */
#define CNF_MAX_HIDDEN 8    /* hidden layers per conditioner MLP            */
#define CNF_MAX_DIM 256     /* logit-vector width D                         */
#define CNF_MAX_WIDTH 512   /* any MLP width                                */

typedef enum cnf_status {
  CNF_OK = 0,
  CNF_ERR_NULL = -1,          /* a required pointer is NULL                   */
  CNF_ERR_DESC = -2,          /* malformed descriptor (dims, abi_version)     */
  CNF_ERR_UNSUPPORTED = -3,   /* shape outside every kernel's envelope        */
  CNF_ERR_BATCH = -4,         /* negative batch                               */
  CNF_ERR_HIP = -5,           /* a HIP launch/copy failed (cnf_last_hip_error) */
  CNF_ERR_ALIGN = -6          /* pointer not 4-byte aligned                   */
} cnf_status;

/* The shape of one Flow made of NvpCouplingLayers (flows/flows.py:68-99). */
typedef struct cnf_desc {
  int32_t abi_version;          /* = CNF_ABI_VERSION                              */
  int32_t dim;                  /* D (n_classes), 2..CNF_MAX_DIM                  */
  int32_t n_layers;             /* L >= 1                                         */
  int32_t n_hidden;             /* len(hidden_size), 0..CNF_MAX_HIDDEN            */
  int32_t hidden[CNF_MAX_HIDDEN];
  int32_t scale;                /* 1: s-net present (RealNVP); 0: NICE, s == 0    */
  int32_t shift;                /* 1: t-net present; 0: t == 0                    */
  int32_t strict_nan;           /* 1: reproduce the reference's inf*0 = NaN at
                                   masked positions (flows/flows.py:107,123)      */
  int32_t options;              /* CNF_OPT_* bits (0: pick the fastest kernel)    */
  const int64_t* perms;         /* HOST pointer, NULL or L*D entries: layer l's
                                   random_flip permutation (flows/flows.py:92-99);
                                   a row whose first entry is < 0 = no perm      */
} cnf_desc;

/* cnf_desc.options: keep a launch off a kernel family (A/B and test use;
 * results agree to fp32 rounding either way). */
#define CNF_OPT_NO_SGPR 1   /* narrow flows: k_valu instead of k_sgpr          */
#define CNF_OPT_NO_WIDE 2   /* wide flows: k_tile instead of k_wide            */
/* Legacy semantics of the reference's TensorFlow flows (code-old/realNVP.py:
 * 19-92; parity unpinned -- TensorFlow is absent):
 *   ALT_MASK  the coupling mask alternates per layer (layer l transforms the
 *             first D//2 features when l is even, the last D//2 when l is
 *             odd) and the data are never flipped (code-old/realNVP.py:66-76);
 *             parameters keep the layer's own column / row order;
 *   S_TANH    the s-net's hidden activations are tanh (code-old/realNVP.py:
 *             58-64); the t-net keeps ReLU.
 * Forward / inverse: k_valu for the narrow shapes of its tables (the code-old
 * default hidden=[dim] at D=3 and 10, and [5,5]), the MFMA-tile family for
 * every other shape; reverse mode: the layer-at-a-time kernels of
 * cnf_wvjp.hip.  Not combinable with random_flip permutations or strict_nan. */
#define CNF_OPT_ALT_MASK 4
#define CNF_OPT_S_TANH 8

/* One float per parameter, in the reference's state_dict order. */
int cnf_param_count(const cnf_desc* desc, int64_t* n_floats);

/* Number of parameter tensors cnf_prepare expects, in this order per layer
 * l = 0..L-1:  [s.layers.0.weight, s.layers.0.bias, ..., s.layers.k.bias]
 * (if scale), then the same for t (if shift).  Weight [out][in] row-major. */
int cnf_param_tensor_count(const cnf_desc* desc, int32_t* n_tensors);

/* Bytes of the device blob cnf_prepare writes (kernel-specific layout). */
int cnf_prepared_bytes(const cnf_desc* desc, size_t* bytes);

/* Reformat the parameters into the blob the selected kernel reads: the mask,
 * the per-layer flip and any random_flip permutation are folded into index
 * tables; weights are restricted to the unmasked block and tiled for the
 * kernel.  params: HOST array of cnf_param_tensor_count DEVICE pointers. */
int cnf_prepare(const cnf_desc* desc, const float* const* params, void* prepared,
                void* stream);

/* Forward + per-sample log-det (Flow.forward):
 *   x      [B][D]      input logits
 *   z      [B][D]      final output (= zs[-1]); may be NULL when z_all != NULL
 *   logdet [B]         sum over layers of sum_j (1-mask_j) s_j; may be NULL
 *   z_all  [L][B][D]   every layer's output (the reference's zs list); may be NULL */
int cnf_forward(const cnf_desc* desc, const void* prepared, const float* x, float* z,
                float* logdet, float* z_all, int64_t B, void* stream);

/* Inverse + log-det (Flow.backward): layers applied L-1..0.
 *   x_all  [L][B][D]   xs list in the reference's order (x_all[L-1] = input
 *                       estimate); may be NULL.  logdet = -(forward log-det). */
int cnf_inverse(const cnf_desc* desc, const void* prepared, const float* z, float* x,
                float* logdet, float* x_all, int64_t B, void* stream);

/* Loss kinds for cnf_forward_loss / cnf_loss_vjp. */
#define CNF_LOSS_CAL 0  /* -mean(log(softmax(z_L)[y] + 1e-7) + ld)   calibrators.py:287-291 */
#define CNF_LOSS_CE 1   /* CE(z_L, y) - det * mean(ld)               run_experiment3D.py:107 */

/* Fused forward + log-det + loss terms (the eval pass of TorchFlowCalibrator.fit,
 * calibrators.py:297-317; the per-step NLL of a sharded batch):
 *   loss_terms[3]  {sum of per-row loss, sum of ce, sum of ld} over the B rows
 *   z, logdet      as cnf_forward, each may be NULL
 * The fused pass writes per-block partial sums into the workspace (no
 * initialisation needed); a one-block follow-up launch adds them in block
 * order (deterministic).  Narrow flows only (sgpr-fused / valu-fused). */
int cnf_forward_loss_workspace_bytes(const cnf_desc* desc, int64_t B, size_t* bytes);
int cnf_forward_loss(const cnf_desc* desc, const void* prepared, const float* x,
                     const int64_t* y, int32_t loss_kind, float det, float* z, float* logdet,
                     float* loss_terms, int64_t B, void* workspace, size_t workspace_bytes,
                     void* stream);

/* Fused calibrated prediction: Calibrator.predict of the flow calibrator
 * (calibrators.py:40-44 with TorchFlowCalibrator.predict_post, :330-353), per row
 *   p = softmax(flow(x - mean(x))),  probs = softmax(log(p + 1e-7) - log_priors)
 *   log_priors [D]     DEVICE pointer (the calibrator's log class priors)
 *   probs      [B][D]  calibrated probabilities
 *   logdet     [B]     log-det of the centred rows, may be NULL
 * Served by k_sgpr (the narrow shapes, random_flip included) and k_wide (the
 * wide shapes of its table, e.g. D=100, hidden [100,100]); CNF_ERR_UNSUPPORTED
 * otherwise (strict_nan, legacy options, other wide shapes: the caller then
 * composes cnf_forward with its own softmax). */
int cnf_predict(const cnf_desc* desc, const void* prepared, const float* x,
                const float* log_priors, float* probs, float* logdet, int64_t B, void* stream);

/* Workspace bytes cnf_vjp / cnf_loss_vjp need for a batch of B rows. */
int cnf_vjp_workspace_bytes(const cnf_desc* desc, int64_t B, size_t* bytes);

/* Reverse mode of cnf_forward (the autograd backward of Flow.forward):
 * given upstream gradients of its outputs, writes
 *   grads  [cnf_param_count]  d/d(parameters), state_dict order (overwritten)
 *   dx     [B][D]             d/dx, may be NULL
 * Upstream inputs, each may be NULL (= zero):
 *   gz     [B][D]     gradient of the final z
 *   gz_all [L][B][D]  gradient of every layer output (the zs list)
 *   gld    [B]        gradient of the per-sample log-det
 * The forward pass is recomputed inside (nothing is saved between calls). */
int cnf_vjp(const cnf_desc* desc, const void* prepared, const float* x, const float* gz,
            const float* gz_all, const float* gld, float* grads, float* dx, int64_t B,
            void* workspace, size_t workspace_bytes, void* stream);

/* Fused forward + loss + reverse mode.  Writes
 *   loss_terms[3]   {sum over rows of the per-row loss, sum of ce, sum of ld}
 *                   (divide by the GLOBAL batch to get the reference's means;
 *                   the split lets data-parallel ranks all-reduce sums)
 *   grads           gradient of (sum over THIS batch of the per-row loss) *
 *                   grad_scale, in cnf_param_count / state_dict order.
 *                   Overwritten, not accumulated.
 *   dx [B][D]       d(loss)/dx, may be NULL
 * Deterministic: no float atomics; fixed-order reductions. */
int cnf_loss_vjp(const cnf_desc* desc, const void* prepared, const float* x,
                 const int64_t* y, int32_t loss_kind, float det, float grad_scale,
                 float* loss_terms, float* grads, float* dx, int64_t B, void* workspace,
                 size_t workspace_bytes, void* stream);

/* Reverse mode of cnf_inverse (autograd through Flow.backward, flows/flows.py:
 * 27-37 / 114-126): given upstream gradients of the inverse's outputs, writes
 *   grads  [cnf_param_count]  d/d(parameters), state_dict order (overwritten)
 *   dz     [B][D]             d/dz, may be NULL
 * Upstream inputs, each may be NULL (= zero):
 *   gx     [B][D]     gradient of the final output (xs[-1], the input estimate)
 *   gx_all [L][B][D]  gradient of every step's output (the xs list, step order)
 *   gld    [B]        gradient of the inverse's per-sample log-det
 * Layer-at-a-time MFMA reverse mode for every shape; strict_nan follows
 * torch autograd's rules for the reference's op sequence (NaN / inf kept). */
int cnf_vjp_inverse_workspace_bytes(const cnf_desc* desc, int64_t B, size_t* bytes);
int cnf_vjp_inverse(const cnf_desc* desc, const void* prepared, const float* z, const float* gx,
                    const float* gx_all, const float* gld, float* grads, float* dz, int64_t B,
                    void* workspace, size_t workspace_bytes, void* stream);

/* One Adam step over every parameter (torch.optim.Adam's update, amsgrad off;
 * the optimizer of TorchFlowCalibrator.fit, calibrators.py:239-295) in one
 * launch, fed by the flat gradient of cnf_loss_vjp / cnf_vjp:
 *   params      HOST array of cnf_param_tensor_count DEVICE pointers, updated
 *               in place (the tensors cnf_prepare reads)
 *   grads       [cnf_param_count]  flat, state_dict order
 *   exp_avg, exp_avg_sq  [cnf_param_count] moments, zero before step 1
 *   step        1-based step count (bias corrections)
 *   lr, beta1, beta2, eps, weight_decay   as the torch optimizer holds them
 *               (Python floats = doubles): 1 - beta, the bias corrections and
 *               lr / (1 - beta1^t) are formed in double and rounded to fp32
 *               once, as torch's scalar arguments are */
int cnf_adam_step(const cnf_desc* desc, float* const* params, const float* grads,
                  float* exp_avg, float* exp_avg_sq, int64_t step, double lr, double beta1,
                  double beta2, double eps, double weight_decay, void* stream);

/* The same step with its two step-dependent scalars read from DEVICE memory,
 * so a HIP graph captured once replays any step (kernel arguments are fixed at
 * capture):  sched[0] = (float)(lr / (1 - beta1^t)),
 *            sched[1] = (float)sqrt(1 - beta2^t)   (formed in double). */
int cnf_adam_step_sched(const cnf_desc* desc, float* const* params, const float* grads,
                        float* exp_avg, float* exp_avg_sq, const float* sched, double beta1,
                        double beta2, double eps, double weight_decay, void* stream);

/* cnf_adam_step (sched == NULL: step and lr as there) or cnf_adam_step_sched
 * (sched != NULL: step and lr ignored) that first reads the DEVICE int32
 * *skip_flag -- the flag cnf_guard_nonfinite ORs into -- and, when it is
 * non-zero, updates nothing: the parameters and both moments keep the last
 * finite step's values, as the reference keeps its weights when it breaks out
 * of the loop before opt.step() on NaN (run_experiment3D.py:129-133).  No host
 * sync: the guard's scan of the gradient and this step queue on one stream. */
int cnf_adam_step_guarded(const cnf_desc* desc, float* const* params, const float* grads,
                          float* exp_avg, float* exp_avg_sq, int64_t step, double lr,
                          const float* sched, double beta1, double beta2, double eps,
                          double weight_decay, const int32_t* skip_flag, void* stream);

/* Device-side non-finite guard (failure detection; the counterpart of the
 * reference's NaN abort, run_experiment3D.py:129-131, without a host sync):
 * scans n floats of a DEVICE array (z, logdet, loss_terms, gradients ...) and
 * ORs into the caller-owned DEVICE int32 *flag:  1 if any element is NaN,
 * 2 if any is +-inf.  The flag is never cleared by the library, so one
 * zeroed flag can accumulate over many launches and be read once.  One
 * HBM-bound pass; an atomic OR only from a wave that found something. */
int cnf_guard_nonfinite(const float* data, int64_t n, int32_t* flag, void* stream);

/* Which kernel family serves this descriptor's launches: "sgpr-fused"
 * (pipelined scalar weights, every output mode), "valu-fused" (strict_nan,
 * shapes whose Linears exceed 32 floats, misaligned views), "mfma-wide"
 * (register-resident MFMA, the wide shapes of its table), "mfma-tile" (other
 * wide shapes, every-layer outputs of wide stacks). */
const char* cnf_kernel_name(const cnf_desc* desc);

const char* cnf_strerror(int status);
/* The hipError_t behind the last CNF_ERR_HIP on this thread. */
int cnf_last_hip_error(void);
int cnf_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* CNF_H_ */
