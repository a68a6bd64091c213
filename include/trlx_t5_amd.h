/*
 * trlx_t5_amd.h — C ABI of the MI355X-native PPO experience-and-loss hot path.
 *
 * Test-free, torch-free boundary: plain device pointers, int64 sizes/strides (in
 * ELEMENTS), dtype enums, scalar hyper-parameters by value and the caller's stream
 * (a hipStream_t passed as void*; NULL = the default stream).  Every entry point is
 * stream-ordered and asynchronous: no host synchronisation, no allocation, no pointer
 * retained past the call.  All return an int status (TRLX_OK = 0); on failure
 * trlx_last_error() returns a thread-local message.
 *
 * The reference (danyang-rainbow/trlx-t5) has no FFI layer: its hot path is plain
 * Python functions.  Each entry point below names the reference function (file:line,
 * into the reference repo) whose arithmetic it replaces; the Python drop-in that binds
 * them (trlx-t5_amd/) keeps those functions' names and signatures.
 *
 * Layout conventions
 *   logits   : [B, T, V], row (b, t) starts at  logits + b*sb + t*st,  V contiguous.
 *   labels   : int64, element (b, t) at labels + b*lb + t*lt, in [0, V) (out of range
 *              produces NaN, never an out-of-bounds read).
 *   [B, T] per-token vectors (logprobs, values, rewards, advantages, ...) : contiguous.
 *   dtype    : TRLX_F32 or TRLX_BF16 (logits / per-token vectors), arithmetic is fp32
 *              with fp64 accumulation for batch statistics.
 */
#ifndef TRLX_T5_AMD_H
#define TRLX_T5_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TRLX_ABI_VERSION 2

typedef enum {
    TRLX_F32 = 0,
    TRLX_BF16 = 1,
    TRLX_I64 = 2,   /* masks / lengths only */
} trlx_dtype;

typedef enum {
    TRLX_OK = 0,
    TRLX_ERR_SHAPE = 1,   /* bad size / shape */
    TRLX_ERR_STRIDE = 2,  /* unsupported stride */
    TRLX_ERR_DTYPE = 3,   /* unsupported dtype */
    TRLX_ERR_LAUNCH = 4,  /* kernel launch failed */
    TRLX_ERR_ARG = 5,     /* NULL pointer / bad scalar */
} trlx_status;

/* Number of fp64 slots per partial-statistics record (see trlx_gae_scan). */
#define TRLX_MOMENT_SLOTS 4     /* {sum x, sum x^2, count, sum mask} */
#define TRLX_SPLIT_MOMENT_SLOTS 8 /* {Σ A0, Σ A0², n, Σ Ak, Σ A0·Ak, Σ Ak², Σ mask, 0} */
/* Number of fp32 slots written by trlx_ppo_loss_finalize (order = stats keys of
 * PPOConfig.loss, ppo_models.py:182-198, after losses). */
#define TRLX_PPO_STATS 13
/* Number of fp64 partial-sum slots per block of trlx_ppo_loss_elem. */
#define TRLX_PPO_PARTIAL_SLOTS 16

int trlx_abi_version(void);
const char* trlx_last_error(void);

/* Launch tuning for A/B measurements (0 = automatic, the default).  The values are
 * thread-local: they steer only the launches issued by the calling host thread, so one
 * thread's experiment never changes another thread's kernels or summation order.  Keys:
 *   "row_variant"       1 = register-resident vocab rows, 2 = streaming vocab rows
 *   "resident_threads"  workgroup size for resident rows (multiple of 64)
 *   "resident_lb512"    1 = <=512-thread resident rows compiled for 8 waves/SIMD (default 0; always on
 *                       for forward rows of <= 8 vectors per thread)
 *   "stream_threads"    workgroup size for streaming rows
 *   "stream_unroll"     16-B loads in flight per thread for streaming rows (2, 4, 8)
 *   "row_order"         resident rows: 0 (default) = step-major vectors, 1 = wave-major
 *   "split_lds"         long rows (fp32 V > 32 k, bf16 V > 32 k): 0 = split VGPR + LDS residency
 *                       for the loss / backward (default), 1 = off, 2 = also for the forward
 *   "split_mid"         mid-length bf16 rows (16k < V <= 32k) in the loss / backward: 0 auto (= 3),
 *                       1 = all in VGPRs, 2 = 5 VGPR + 3 LDS vector steps, 3 = 6 + 2 (8 waves/SIMD)
 *   "ragged_order"      ragged experience rows with an order scratch: 0 = valid rows first (default),
 *                       1 = natural order
 *   "order_launch"      the valid-rows-first order: 0 auto (one launch up to 64 chunks of 1024 rows,
 *                       then two), 1 = one launch, 2 = two chunk-count launches
 *   "lmloss_splits"     fused loss forward vocab splits: 0 auto (the fullest last round), 1..8 fixed
 *   "lmloss_dw_tsplit"  fused loss dW: 0 auto (the last round's vocab blocks split over the tokens),
 *                       1 = no split, 2..16 = that many token splits
 *   "lmloss_fwd"        fused loss forward form: 0 / 2 = the 16x16x32 form (the only one built; the
 *                       removed forms 1, 3, 4 are rejected with TRLX_ERR_ARG)
 *   "lmloss_dw"         fused loss dW plan: 0 auto (saved P where the caller's buffers hold it),
 *                       1 = recompute S (k_lmloss_dw), 4 = saved P (k_lmloss_dwp); 2, 3 rejected
 *   "lmloss_dwp_form"   saved-P dW blocking: 0 auto (= 2: 32 rows a wave x H/2), 1 = 16 rows a wave x H
 *   "store_policy"      gradient-row store cache policy: 0 auto (default: nt; sc1 for all-VGPR rows
 *                       launches writing > 1.5 GB), 1 none, 2 sc1, 3 sc0|sc1, 4 nt|sc1, 5 nt
 * Results are identical up to fp32 summation order; only speed changes. */
int trlx_set_tuning(const char* key, int64_t value);

/* ---------------------------------------------------------------- A1
 * logprobs_from_logits forward — replaces trlx/utils/modeling.py:37-41
 * (F.log_softmax over V + gather at labels), fused in one pass over each row; the
 * [B,T,V] log-softmax is never materialised.
 * Up to two logits tensors of identical shape/strides/dtype are processed in one launch
 * (x1 may be NULL): the experience step's policy and reference logits
 * (ppo_orchestrator.py:154-155).  out_lp{0,1}: [B,T] of out_dtype.  out_lse{0,1}:
 * optional fp32 [B,T] log-sum-exp saved for the backward. */
int trlx_lsm_gather_fwd(const void* x0, const void* x1, int dtype,
                        int64_t B, int64_t T, int64_t V, int64_t sb, int64_t st,
                        const int64_t* labels, int64_t lb, int64_t lt,
                        void* out_lp0, void* out_lp1, int out_dtype,
                        float* out_lse0, float* out_lse1, void* stream);
/* The experience rows of a ragged batch (decoder lengths [B] int64): a row (b, t) with
 * t >= lengths[b] is store padding — ppo_pipeline.py:47-65 pads each element's logprobs with
 * 0.0 — so its lp is 0 and the row is NOT read (the bytes of a batch of decoder lengths L_b
 * are those of its sum(L_b) tokens).  lengths == NULL: trlx_lsm_gather_fwd.  order_ws (or
 * NULL): trlx_ragged_order_bytes(B, T) bytes of device scratch — a small launch
 * first orders the rows valid-first so the skipped rows do not interleave with them (the
 * scratch then holds the B·T row ids, valid first and ~id for the padding, and the count). */
int64_t trlx_ragged_order_bytes(int64_t B, int64_t T);
int trlx_lsm_gather_fwd_ragged(const void* x0, const void* x1, int dtype,
                               int64_t B, int64_t T, int64_t V, int64_t sb, int64_t st,
                               const int64_t* labels, int64_t lb, int64_t lt, const int64_t* lengths,
                               void* order_ws, void* out_lp0, void* out_lp1, int out_dtype, void* stream);

/* ---------------------------------------------------------------- A1 backward
 * Autograd of modeling.py:39-40 (log_softmax_backward of the gathered one-hot):
 *   dx[b,t,j] = g[b,t] * ([j == y] - exp(x[b,t,j] - lse[b,t]))
 * grad: [B,T] of grad_dtype; dx row (b,t) at dx + b*dsb + t*dst, same dtype as x.  One
 * read of the row and one write, no reduction (lse from the forward). */
int trlx_lsm_gather_bwd(const void* x, int dtype, int64_t B, int64_t T, int64_t V,
                        int64_t sb, int64_t st, const int64_t* labels, int64_t lb, int64_t lt,
                        const float* lse, const void* grad, int grad_dtype,
                        void* dx, int64_t dsb, int64_t dst, void* stream);

/* ---------------------------------------------------------------- A2
 * KL-penalised reward — replaces ppo_orchestrator.py:164-167:
 *   r[b,t] = -beta * (lp[b,t] - ref_lp[b,t]);  r[b, T-1] += scores[b]
 * (with lengths != NULL the score goes to column lengths[b]-1 and columns >= lengths[b]
 * are padding: reward 0).  lp/ref_lp: [B,T] of in_dtype; scores fp32 [B] or NULL. */
int trlx_kl_penalty_rewards(const void* lp, const void* ref_lp, int in_dtype,
                            int64_t B, int64_t T, float beta, const float* scores,
                            const int64_t* lengths, void* rewards, int out_dtype, void* stream);

/* ---------------------------------------------------------------- A5 (+A2 fused, +A3 partials)
 * GAE reverse scan — replaces ppo_models.py:121-136 (the per-t Python loop):
 *   delta_t = r_t + gamma*V_{t+1} - V_t   (V_T := 0);   A_t = delta_t + (gamma*lam)*A_{t+1}
 *   returns = A + V  (unwhitened A)
 * values / rewards: [B, T] of dtype (rows contiguous, row stride T); columns
 * [0, Teff) are used (Teff = response_length).  If lp != NULL the rewards are not read
 * but computed in-kernel from (lp, ref_lp, neg_beta, scores) exactly as
 * trlx_kl_penalty_rewards does (fp32 lp/ref_lp [B,T]) and, if rew_out != NULL, stored.
 * lengths (nullable): positions t >= lengths[b] are padding (value/reward read as 0).
 * Outputs: adv_raw fp32 [B,Teff] (unwhitened), ret [B,Teff] of ret_dtype, and per-block
 * partial moments of adv_raw: partials[blk*4 + {0,1,2,3}] = {sum A, sum A^2, count,
 * sum mask} (mask: int64 [B,Teff] loss mask, NULL = all ones).
 * trlx_gae_num_blocks(B, Teff) tells how many partial records are written.  With
 * stats != NULL the last block to finish also reduces them (fixed order) into stats[4];
 * `ticket` is then a device uint32 that must be 0 before the first call (the kernel
 * re-arms it). */
int64_t trlx_gae_num_blocks(int64_t B, int64_t Teff);
int trlx_gae_scan(const void* values, const void* rewards, int dtype, int64_t B, int64_t T,
                  int64_t Teff, float gamma, float lam,
                  const float* lp, const float* ref_lp, float neg_beta, const float* scores,
                  const int64_t* lengths, const int64_t* mask,
                  float* adv_raw, void* ret, int ret_dtype, void* rew_out, int rew_dtype,
                  double* partials, double* stats, unsigned* ticket, void* stream);

/* ---------------------------------------------------------------- A3 helpers
 * Partial moments of an arbitrary contiguous tensor (for whiten / get_global_statistics,
 * modeling.py:9-34, and RunningMoments, :72-104).  trlx_moments_num_blocks(n) records. */
int64_t trlx_moments_num_blocks(int64_t n);
int trlx_moments_partial(const void* x, int dtype, int64_t n, double* partials, void* stream);
/* (dtype may also be TRLX_I64 here, e.g. to sum a loss mask.) */
/* Reduce nblk partial records (fixed order, deterministic) into stats[4]. */
int trlx_moments_finalize(const double* partials, int64_t nblk, double* stats, void* stream);

/* ---------------------------------------------------------------- A4
 * whiten — replaces modeling.py:24-34:  out = (x - mu) * rsqrt(var + 1e-8) [+ mu]
 * mu, var from stats[4] = {sum, sumsq, count, .}: var = M2/count (biased, the
 * distributed branch) or M2/(count-1) (unbiased, torch.var_mean branch). */
int trlx_whiten_apply(const void* x, int dtype, int64_t n, const double* stats, int unbiased,
                      int shift_mean, void* out, int out_dtype, void* stream);

/* ---------------------------------------------------------------- A1+A4+A6 fused (loss side)
 * One pass over each policy-logits row: lse, lp = x[y] - lse, then the closed-form
 * per-token gradient of PPOConfig.loss's policy term (ppo_models.py:165-177 with torch's
 * max-tie and clamp-bound rules) and the row's dlogits = g * (onehot - softmax), written
 * once.  Advantages are whitened on the fly from adv_raw + stats (stats == NULL: adv is
 * used as given).  mask: int64 [B,T] or NULL (all ones); msum: device fp64 scalar (NULL:
 * use msum_host).  Outputs: lp_out fp32 [B,T]; dx (row (b,t) at dx + b*dsb + t*dst, dtype
 * of x).  A masked token (mask == 0) has d loss / d lp = 0 exactly, so its dlogits row is
 * written as zeros WITHOUT reading its logits and lp_out is 0 there (for every loss-rows
 * entry point below as well; the token's loss terms are those of any finite lp). */
int trlx_ppo_policy_fused(const void* x, int dtype, int64_t B, int64_t T, int64_t V,
                          int64_t sb, int64_t st, const int64_t* labels, int64_t lb, int64_t lt,
                          const void* old_lp, int old_dtype, const float* adv,
                          const double* stats, int unbiased, const int64_t* mask,
                          const double* msum, double msum_host, float cliprange,
                          float* lp_out, void* dx, int64_t dsb, int64_t dst, void* stream);

/* ---------------------------------------------------------------- the fused step (2 launches)
 * Experience: policy + reference rows -> lp, ref_lp (fp32); then one wavefront per rollout
 * computes its KL-penalised rewards, GAE advantages (unwhitened, fp32) and returns, and the
 * last block the whitening moments stats[4] = {Σ A, Σ A², n, Σ mask}.  Replaces ppo_orchestrator.py:
 * 154-167 followed by ppo_models.py:121-136 (+ the moments of modeling.py:24-29).
 * Loss: new-policy rows -> lp_out, dlogits (one read + one write), the value-loss gradient
 * dvalues and per-token loss terms; then one wavefront per rollout sums them and the last
 * block writes loss[1] + loss_stats[13] (order of trlx_ppo_loss_finalize),
 * i.e. ppo_models.py:141-199 with its autograd into the logits.  `stats` (possibly
 * all-reduced across ranks in between) whitens the advantages on the fly; unbiased as in
 * trlx_whiten_apply.  workspace: trlx_ppo_workspace_bytes(B, T) bytes, zero-filled once
 * before the first use and then reusable (the kernels re-arm their tickets).  Rows (b, t)
 * of the rollout batch must be contiguous rollouts (t fastest).  With lengths, the
 * experience rows past each rollout's length are store padding (lp = ref_lp = 0, not read:
 * trlx_lsm_gather_fwd_ragged); with a mask, the loss rows of masked tokens are not read
 * (trlx_ppo_policy_fused). */
int64_t trlx_ppo_workspace_bytes(int64_t B, int64_t T);
int trlx_ppo_experience_fused(const void* logits, const void* ref_logits, int dtype, int64_t B, int64_t T,
                              int64_t V, int64_t sb, int64_t st, const int64_t* labels, int64_t lb,
                              int64_t lt, const void* values, int v_dtype, const float* scores,
                              const int64_t* lengths, const int64_t* mask, float kl_coef, float gamma,
                              float lam, float* lp, float* ref_lp, float* rewards, float* adv_raw,
                              void* ret, int ret_dtype, double* stats, void* workspace, void* stream);
/* The two launches of each fused entry point, separately (same arguments):
 *   experience = trlx_lsm_gather_fwd_ragged(policy, ref -> fp32 lp, ref_lp) + trlx_ppo_rollout_gae
 *   loss       = trlx_ppo_loss_rows + trlx_ppo_rollout_loss  */
int trlx_ppo_rollout_gae(int64_t B, int64_t T, const float* lp, const float* ref_lp, const void* values,
                         int v_dtype, const float* scores, const int64_t* lengths, const int64_t* mask,
                         float kl_coef, float gamma, float lam, float* rewards, float* adv_raw, void* ret,
                         int ret_dtype, double* stats, void* workspace, void* stream);
int trlx_ppo_loss_rows(const void* logits, int dtype, int64_t B, int64_t T, int64_t V, int64_t sb, int64_t st,
                       const int64_t* labels, int64_t lb, int64_t lt, const void* old_lp, int old_dtype,
                       const float* adv_raw, const double* stats, int unbiased, const int64_t* mask,
                       const void* values, int v_dtype, const void* old_values, int ov_dtype,
                       const void* returns, int r_dtype, float cliprange, float cliprange_value, float vf_coef,
                       float* lp_out, void* dx, int64_t dsb, int64_t dst, float* dvalues, void* workspace,
                       void* stream);
int trlx_ppo_rollout_loss(int64_t B, int64_t T, const double* stats, float vf_coef, float* loss,
                          float* loss_stats, void* workspace, void* stream);
int trlx_ppo_loss_fused(const void* logits, int dtype, int64_t B, int64_t T, int64_t V, int64_t sb,
                        int64_t st, const int64_t* labels, int64_t lb, int64_t lt, const void* old_lp,
                        int old_dtype, const float* adv_raw, const double* stats, int unbiased,
                        const int64_t* mask, const void* values, int v_dtype, const void* old_values,
                        int ov_dtype, const void* returns, int r_dtype, float cliprange,
                        float cliprange_value, float vf_coef, float* lp_out, void* dx, int64_t dsb,
                        int64_t dst, float* dvalues, float* loss, float* loss_stats, void* workspace,
                        void* stream);

/* ---------------------------------------------------------------- A6
 * PPOConfig.loss (ppo_models.py:141-199) over [B,T] vectors.  Pass 1 (elementwise,
 * many blocks): per-token value/policy terms, gradients d loss/d lp (dlp, optional) and
 * d loss/d values (dv, optional) and fp64 partial sums (TRLX_PPO_PARTIAL_SLOTS per
 * block).  Pass 2 (one block, fixed order): loss[1] and stats[TRLX_PPO_STATS] fp32 in the
 * order total_loss, policy_loss, value_loss, mean_old_values, var_old_values,
 * mean_values, values_error, values_clipfrac, approx_kl, policy_clipfrac,
 * returns_mean, returns_var, ratio.
 * lp, values, old_lp, old_values, adv, returns: [n] of the respective dtypes (adv fp32,
 * optionally whitened on the fly from adv_stats); mask int64 [n] or NULL. */
int64_t trlx_ppo_loss_num_blocks(int64_t n);
int trlx_ppo_loss_elem(int64_t n, const void* lp, int lp_dtype, const void* values, int v_dtype,
                       const void* old_lp, int olp_dtype, const void* old_values, int ov_dtype,
                       const void* adv, int a_dtype,
                       const double* adv_stats, int unbiased, const void* returns,
                       int r_dtype, const int64_t* mask, const double* msum, double msum_host,
                       float cliprange, float cliprange_value, float vf_coef,
                       void* dlp, void* dv, int g_dtype, double* partials,
                       float* loss, float* stats, unsigned* ticket, void* stream);
/* (with ticket != NULL — a device uint32, 0 before the first call — the last block of
 *  trlx_ppo_loss_elem performs pass 2 itself: one launch for the whole loss.) */
int trlx_ppo_loss_finalize(const double* partials, int64_t nblk, int64_t n,
                           const double* msum, double msum_host, float vf_coef,
                           float* loss, float* stats, void* stream);

/* ---------------------------------------------------------------- A10 (ILQL loss)
 * ILQLConfig.loss — replaces trlx/model/nn/ilql_models.py:52-116 with its autograd
 * (config 5).  Every vocab row (logits [B,L,V] and the nq Q-head rows [B,A,V]) is read
 * once into registers and its gradient row written once:
 *   logits row (b,t<L-1): CE against input_ids[b,t+1], weight attention_mask[b,t+1]
 *                         (AWAC, :98-105); row t = L-1 gets a zero gradient
 *   q_i row (b,a)       : CE against the action a* = input_ids[b, 1+actions_ixs[b,a]]
 *                         weighted by dones[b,a] (CQL, :87-96) + the TD term
 *                         ((Q_i[a*] - (r + gamma*vs[b,a+1]*dones[b,a+1]))*dones[b,a])^2 (:63-74)
 *   target-Q rows are only gathered at a* (min over heads) for the expectile V loss (:76-83).
 * Three launches: prep (n_nonterminal = max(1, sum dones[:, :-1]) and sum attention[:, 1:]),
 * rows (one workgroup per vocab row), finalize (fixed-order fp64 sums -> losses[5] =
 * {loss, loss_q, loss_v, loss_cql, loss_awac}); prep and finalize run a few workgroups whose
 * last reduces the block records in fixed order (an arrival ticket in the workspace).  dvs = d loss / d vs (fp32 [B, A+1], last
 * column 0).  Gradient rows have the same strides and 16-B phase as their inputs.  The
 * small [B, .] tensors are contiguous.  No collective: the reference's ILQL loss is
 * rank-local (DDP averages the gradients). */
typedef struct {
    int dtype;                        /* TRLX_F32 / TRLX_BF16: logits, q, tq rows */
    int nq;                           /* 1 or 2 Q heads (ILQLConfig.two_qs) */
    int64_t B, L, A, V;               /* rows, tokens, actions (states = A + 1), vocab */
    const void* logits;               /* [B,L,V], row (b,t) at logits + b*logits_sb + t*logits_st */
    int64_t logits_sb, logits_st;
    const void* q[2];                 /* [B,A,V] Q heads (q[1] unused when nq == 1) */
    int64_t q_sb[2], q_st[2];
    const void* tq[2];                /* [B,A,V] target Q heads (gathered only) */
    int64_t tq_sb[2], tq_st[2];
    const int64_t* input_ids;         /* [B,L] */
    const int64_t* attention_mask;    /* [B,L] */
    const int64_t* actions_ixs;       /* [B,A] */
    const int64_t* dones;             /* [B,A+1] */
    const void* rewards;              /* [B,A] */
    int rewards_dtype;
    const void* vs;                   /* [B,A+1] (the reference's [B,S,1]) */
    int vs_dtype;
    float tau, gamma, cql_scale, awac_scale;
    void* dlogits;                    /* gradient rows, dtype of the inputs */
    int64_t dlogits_sb, dlogits_st;
    void* dq[2];
    int64_t dq_sb[2], dq_st[2];
    float* dvs;                       /* [B,A+1] fp32 */
    float* losses;                    /* [5] fp32 */
    void* workspace;                  /* trlx_ilql_workspace_bytes(B, L, A, nq) bytes, zero-filled
                                         once before first use (prep / finalize re-arm their tickets) */
} trlx_ilql_args;

int64_t trlx_ilql_workspace_bytes(int64_t B, int64_t L, int64_t A, int nq);
int trlx_ilql_prep(const trlx_ilql_args* args, void* stream);
int trlx_ilql_rows(const trlx_ilql_args* args, void* stream);
int trlx_ilql_finalize(const trlx_ilql_args* args, void* stream);
int trlx_ilql_loss_fused(const trlx_ilql_args* args, void* stream);   /* the three in order */

/* ---------------------------------------------------------------- §8f rank 2: fused lm_head + logprobs
 * lp[n] = h[n]·W[y_n] − logsumexp_v h[n]·W[v] without materialising the [N, V] logits —
 * replaces `logits = lm_head(hs)` (ppo_models.py:640 T5HeadWithValueModel, :274/:588 GPT)
 * + logprobs_from_logits (modeling.py:37-41) on the experience side
 * (ppo_orchestrator.py:135-155, no gradient).  hidden: bf16 [N, H] rows of ldh elements;
 * weight: bf16 [V, H] (nn.Linear layout) rows of ldw; H a multiple of 64, rows 16-B
 * aligned.  labels int64 (stride lb; out of range -> NaN).  lp_out [N] of lp_dtype
 * (F32/BF16), lse_out optional fp32 [N].  MFMA (bf16 in, fp32 accumulate) tiles of
 * 256 tokens x 256 vocab (128 x 128 for small N) with an online max/Σexp epilogue, then a
 * per-token combine.
 * workspace: trlx_lmhead_workspace_bytes(N, V) bytes (no initialisation needed). */
int64_t trlx_lmhead_workspace_bytes(int64_t N, int64_t V);
/* Kernel variant (0 = automatic: 8 for N >= 2048, else 3; 3 = 128x128 tiles, 2 barriers per
 * K-step; 8 = 256x256 ping-pong, two wave groups staggered by a barrier, 2 phases per K-step).
 * Other values are rejected (the round-1 variants that measured slower were removed).  Results
 * identical up to fp32 summation order.  Set before sizing the workspace (the vocab tile width
 * changes it). */
int trlx_lmhead_set_variant(int variant);
int trlx_lmhead_logprobs(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                         int64_t H, int64_t V, const int64_t* labels, int64_t lb, void* lp_out,
                         int lp_dtype, float* lse_out, void* workspace, void* stream);
/* The same over a ragged batch: N = B·T tokens in rollouts of T, decoder lengths [B] int64.
 * Tokens past their rollout's length are store padding: lp (and lse) 0 there.  With an order
 * scratch (trlx_ragged_order_bytes(B, T) bytes) the 128 x 256 MFMA tiles (the H <= 1024,
 * N >= 2048 variant) gather the valid tokens' hidden rows and skip the padding's tiles — the
 * GEMM work of a batch of decoder lengths L_b is that of its sum(L_b) tokens; the other
 * variants compute every token and zero the padding's lp.  N·ldh·2 must stay below 2 GB. */
int trlx_lmhead_logprobs_ragged(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                                int64_t H, int64_t V, const int64_t* labels, int64_t lb, const int64_t* lengths,
                                int64_t T, void* order_ws, void* lp_out, int lp_dtype, float* lse_out,
                                void* workspace, void* stream);

/* ---------------------------------------------------------------- §8f rank 2, loss side: fused lm_head fwd + bwd
 * The policy update's lm_head (ppo_models.py:640 T5, :274 GPT) + logprobs_from_logits
 * (modeling.py:37-41) + autograd back through both (accelerate_ppo_model.py:96-118), with the
 * [N, V] logits and dlogits never written: with p = softmax(h·Wᵀ) and g = d loss / d lp,
 *   dh_t = g_t·(W[y_t] − Σ_v p_tv·W_v)      dW_v = Σ_t g_t·(1[y_t = v] − p_tv)·h_t.
 * hidden [N, ldh] bf16 (N = B·T tokens, row t of rollout b = token b·T + t), weight [V, ldw]
 * bf16 (nn.Linear layout), H in {512, 768}; dweight [V, lddw] of dw_dtype (overwritten); dhidden
 * [N, lddh] of dh_dtype (bf16 / fp32, lddh a multiple of 4).  Three MFMA launches + small
 * ones: a flash-style forward (online softmax and O = Σ_v P·W_v per token and vocab split), a
 * per-token combine (lse, lp, g, dh) and a dW pass that recomputes each logits tile and
 * accumulates dSᵀ·h — or, in the PPO entries given the larger saved-P workspace, reads the
 * forward's bf16 P tiles back instead of recomputing them; deterministic (fixed-order sums, no
 * atomics).
 * lm_workspace: trlx_lmhead_loss_workspace_bytes(N, H, V) bytes, no initialisation. */
int64_t trlx_lmhead_loss_workspace_bytes(int64_t N, int64_t H, int64_t V);
/* The PPO entries' workspace with room for the saved-P plan (the forward's bf16 P tiles,
 * ⌈V/64⌉·2⌈N/64⌉·4 KB: 0.62 GB at N = 6144, V = 50257, plus per-(split, token) records).  Pass
 * its size as lm_workspace_bytes; a workspace of only trlx_lmhead_loss_workspace_bytes runs the
 * recompute plan. */
int64_t trlx_ppo_loss_from_hidden_workspace_bytes(int64_t N, int64_t H, int64_t V);
/* The plan the PPO entries run for this shape and workspace size: 1 = saved P (three MFMA
 * passes: S and O forward, dSᵀ·h from the stored P), 0 = recompute (four: S recomputed in dW). */
int trlx_ppo_loss_from_hidden_plan(int64_t N, int64_t H, int64_t V, int64_t lm_workspace_bytes);
/* The smaller workspace trlx_lmhead_logprobs_bwd / _bwd_savep need (no forward partials). */
int64_t trlx_lmhead_loss_bwd_workspace_bytes(int64_t N, int64_t H, int64_t V);
/* The PPO loss from the policy's last hidden states: trlx_ppo_loss_rows's arguments with the
 * logits replaced by (hidden, weight) and dlogits by (dhidden, dweight) — same token records
 * in `workspace` (trlx_ppo_rollout_loss then emits loss + stats), same whitening of adv_raw by
 * `stats` (NULL: adv_raw used as given, and then only mask = NULL: the loss normaliser Σ mask
 * is read at stats[3]), dvalues, lp_out.  Tokens with mask == 0 are skipped (compacted out of
 * all three MFMA passes: zero gradient, lp_out 0, their token records as the masked loss rows
 * write them).  N·ldh·2 and V·ldw·2 must stay below 2 GB (32-bit tile addressing).
 * lm_workspace_bytes: the size of lm_workspace (>= trlx_lmhead_loss_workspace_bytes, else
 * TRLX_ERR_ARG; >= trlx_ppo_loss_from_hidden_workspace_bytes selects the saved-P plan). */
int trlx_ppo_loss_from_hidden(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t B,
                              int64_t T, int64_t H, int64_t V, const int64_t* labels, const void* old_lp,
                              int old_dtype, const float* adv_raw, const double* stats, int unbiased,
                              const int64_t* mask, const void* values, int v_dtype, const void* old_values,
                              int ov_dtype, const void* returns, int r_dtype, float cliprange,
                              float cliprange_value, float vf_coef, float* lp_out, void* dhidden, int64_t lddh,
                              int dh_dtype, void* dweight, int dw_dtype, int64_t lddw, float* dvalues,
                              void* workspace, void* lm_workspace, int64_t lm_workspace_bytes, void* stream);
/* The split-beta form (the pipelined data-parallel schedule; see trlx_ppo_loss_rows_split /
 * trlx_ppo_loss_rows_split_gae): the advantage A0 - beta*Ak whitened by coefficients that are
 * either given (`coef`, stored by an earlier loss on the same experience) or derived here from
 * the all-reduced split record `stats8` and beta (ctl_state[TRLX_CTL_KL_COEF], or kl_coef when
 * ctl_state is NULL; `unbiased` as there) and stored to coef_out (may be NULL) — exactly one of
 * coef / stats8.  The batch's rewards and returns (r_dtype) are written here; msum = Σ mask
 * (stats8 + 6; required with a mask); the loss tail takes stats8 + 3 as its `stats`. */
int trlx_ppo_loss_from_hidden_split(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t B,
                                    int64_t T, int64_t H, int64_t V, const int64_t* labels, const void* old_lp,
                                    int old_dtype, const float* adv0, const float* adv_kl, const float* rew_kl,
                                    const float* rew_score, const float* coef, const double* stats8, int unbiased,
                                    const double* ctl_state, float kl_coef, float* coef_out, const double* msum,
                                    const int64_t* mask, const void* values, int v_dtype, const void* old_values,
                                    int ov_dtype, float* rewards, void* returns, int r_dtype, float cliprange,
                                    float cliprange_value, float vf_coef, float* lp_out, void* dhidden, int64_t lddh,
                                    int dh_dtype, void* dweight, int dw_dtype, int64_t lddw, float* dvalues,
                                    void* workspace, void* lm_workspace, int64_t lm_workspace_bytes,
                                    void* stream);
/* The differentiable building block (logprobs_from_logits(lm_head(h), y) with autograd):
 * forward -> lp [N] (lp_dtype), lse [N] fp32 and E = Σ_v p_tv·W_v [N, H] fp32 (saved for the
 * backward); backward(grad = d loss / d lp [N], F32 / BF16) -> dhidden, dweight (either may be
 * NULL: a frozen lm_head skips the dW pass; lm_workspace: trlx_lmhead_loss_bwd_workspace_bytes). */
int trlx_lmhead_logprobs_fwd_saved(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                                   int64_t H, int64_t V, const int64_t* labels, int64_t lb, void* lp_out,
                                   int lp_dtype, float* lse_out, float* e_out, void* lm_workspace, void* stream);
int trlx_lmhead_logprobs_bwd(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                             int64_t H, int64_t V, const int64_t* labels, int64_t lb, const void* grad,
                             int grad_dtype, const float* lse, const float* e, void* dhidden, int64_t lddh,
                             int dh_dtype, void* dweight, int dw_dtype, int64_t lddw, void* lm_workspace,
                             void* stream);
/* The same pair, extended (replaces the same reference lines as the pair above:
 * accelerate_ppo_model.py:96-118 through ppo_models.py:640 and modeling.py:37-41):
 *   saved: NULL = the recompute plan (as above), or a region of trlx_lmhead_savep_bytes(N, H, V)
 *          bytes (⌈V/64⌉·2⌈N/64⌉·4 KB + 128·N B: 0.62 GB at N = 6144, V = 50257 — the size of
 *          bf16 logits) the forward fills with its bf16 P tiles and per-(split, token) records
 *          and the caller keeps, unmodified, until the backward: the dW pass then reads P back
 *          (3 MFMA passes in all) instead of recomputing S (4);
 *   mask:  NULL = every token, or [N] int64: tokens with mask == 0 are compacted out of every
 *          MFMA pass — their lp and lse are 0 and they get a zero dh and no share of dW (what the
 *          PPO loss's own mask gives them: ppo_models.py:150-199 multiplies every lp term by it).
 *          The backward takes the same mask (it rebuilds the same stable order).
 * The "lmloss_splits" tuning must not change between the two calls (the records follow the
 * forward's split plan).  lm_workspace as the pair above. */
int64_t trlx_lmhead_savep_bytes(int64_t N, int64_t H, int64_t V);
int trlx_lmhead_logprobs_fwd_ex(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                                int64_t H, int64_t V, const int64_t* labels, int64_t lb, const int64_t* mask,
                                void* lp_out, int lp_dtype, float* lse_out, float* e_out, void* lm_workspace,
                                void* saved, void* stream);
int trlx_lmhead_logprobs_bwd_ex(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                                int64_t H, int64_t V, const int64_t* labels, int64_t lb, const int64_t* mask,
                                const void* grad, int grad_dtype, const float* lse, const float* e, void* dhidden,
                                int64_t lddh, int dh_dtype, void* dweight, int dw_dtype, int64_t lddw,
                                void* lm_workspace, const void* saved, void* stream);

/* ---------------------------------------------------------------- §8f rank 3: ILQL sampling step
 * One decode step of CausalLMWithValueHeads.generate (ilql_models.py:296-316) per row b:
 *   score = log_softmax(logits[b]) + beta*(min(tq0[b], tq1[b]) - vs[b])  (logits -inf where
 *   logit_mask[prev_ids[b]] is set), topk_mask(score, top_k) (:24-28, ties at the threshold
 *   kept), pi = softmax(. / temperature); out_ids[b] = the inverse CDF of pi at u[b] (index
 *   order; u from the caller's generator replaces torch.multinomial's draw);
 *   out = finished ? eos : out; finished = out == eos.
 * logits / tq rows: [B, V] of dtype with row strides ld_*; tq1 may be NULL (one head);
 * logit_mask: NULL or uint8 [*, V] rows of ld_mask; finished: int64 [B] in/out or NULL. */
int trlx_ilql_sample(const void* logits, int64_t ld_logits, const void* tq0, int64_t ld_tq0,
                     const void* tq1, int64_t ld_tq1, int dtype, const float* vs,
                     const uint8_t* logit_mask, int64_t ld_mask, const int64_t* prev_ids, int64_t B,
                     int64_t V, float beta, int top_k, float temperature, const float* u,
                     int64_t* out_ids, int64_t* finished, int64_t eos, void* stream);

/* ---------------------------------------------------------------- §8f: device-resident rollout store
 * Row copy between padded columnar [rows, W] buffers — replaces the reference's
 * `.cpu()` of the experience tensors, per-sample PPORLElement lists and the pad_sequence
 * collate (ppo_orchestrator.py:169-187, ppo_pipeline.py:36-66).  For each of nfields
 * (<= 8) fields i, for j < rows and c < cols[i]:
 *   dst[i][drow(j) * dst_ld[i] + dst_col0[i] + c] = src[i][srow(j) * src_ld[i] + src_col0[i] + c]
 * srow(j) = src_idx ? src_idx[j] : src_row0 + j (drow likewise); element size esize[i] in
 * {2, 4, 8} bytes; strides / columns in elements.  The host arrays are read during the call
 * only; src_idx / dst_idx are device int64 vectors. */
int trlx_rows_copy(int nfields, const void* const* src, void* const* dst, const int64_t* src_ld,
                   const int64_t* dst_ld, const int64_t* src_col0, const int64_t* dst_col0,
                   const int64_t* cols, const int* esize, int64_t rows, const int64_t* src_idx,
                   int64_t src_row0, const int64_t* dst_idx, int64_t dst_row0, void* stream);

/* decoder_input_ids of the seq2seq policy forward from a collated response batch — replaces
 * shift_tokens_right (trlx/model/accelerate_ppo_model.py:18-25) as called by
 * AcceleratePPOModel.get_model_inputs (:63-76): out[b,0] = decoder_start_token_id,
 * out[b,t] = ids[b,t-1], then every -100 -> pad_token_id.  ids / out: device int64 [B, T] with
 * row strides ld / out_ld (unit column stride), out must not alias ids; T >= 1 (the reference
 * raises IndexError on an empty response), B = 0 is a no-op. */
int trlx_shift_tokens_right(const int64_t* ids, int64_t B, int64_t T, int64_t ld, int64_t pad_token_id,
                            int64_t decoder_start_token_id, int64_t* out, int64_t out_ld, void* stream);

/* ---------------------------------------------------------------- §8f rank 4: device-resident controller state
 * The PPO loop's host scalars — RunningMoments of the scores (trlx/utils/modeling.py:72-104),
 * the orchestrator's ref_mean/ref_std + score scale/clip (ppo_orchestrator.py:48-49,96-112)
 * and the KL coefficient of Adaptive/FixedKLController (ppo_models.py:26-58) — as ONE fp64
 * record in device memory, read and advanced in-stream (no host synchronisation).
 * Slots (doubles): */
#define TRLX_CTL_SLOTS 16
#define TRLX_CTL_MEAN 0          /* RunningMoments.mean  */
#define TRLX_CTL_VAR 1           /* RunningMoments.var   */
#define TRLX_CTL_STD 2           /* RunningMoments.std   */
#define TRLX_CTL_COUNT 3         /* RunningMoments.count */
#define TRLX_CTL_REF_MEAN 4      /* orchestrator ref_mean */
#define TRLX_CTL_REF_STD 5       /* orchestrator ref_std  */
#define TRLX_CTL_REF_SET 6       /* 1 once ref_mean is known (config or first batch) */
#define TRLX_CTL_KL_COEF 7       /* kl_ctl.value (beta) */
#define TRLX_CTL_BATCH_MEAN 8    /* last RunningMoments.update return values */
#define TRLX_CTL_BATCH_STD 9
#define TRLX_CTL_KL_UPDATES 10   /* number of kl_ctl.update calls */
#define TRLX_CTL_LAST_KL 11      /* last approx_kl given to kl_ctl.update */

typedef enum {
    TRLX_SCALE_NONE = 0,     /* scale_reward False */
    TRLX_SCALE_RUNNING = 1,  /* "running": scores /= running.std */
    TRLX_SCALE_REF = 2,      /* "ref": scores /= ref_std */
} trlx_scale_mode;

/* Score-side control: RunningMoments.update(scores) (global moments when given: the
 * all-reduced {Σx, Σx², n} of trlx_score_moments over ranks, else the local batch), the
 * first-batch ref_mean/ref_std, then scores = clip(scores / scale, ±cliprange_reward). */
typedef struct {
    const double* state_in;          /* [TRLX_CTL_SLOTS] */
    double* state_out;               /* [TRLX_CTL_SLOTS], may equal state_in only in trlx_score_ctl_update */
    const double* global_moments;    /* [>=3] or NULL */
    int scale_mode;                  /* trlx_scale_mode */
    float cliprange_reward;          /* 0 = no clip */
} trlx_score_ctl;

/* KL-side control: kl_ctl.update(approx_kl, n_steps) on state (in place). */
typedef struct {
    double* state;                   /* [TRLX_CTL_SLOTS] */
    int adaptive;                    /* 1 AdaptiveKLController, 0 FixedKLController */
    double target, horizon;
    int64_t n_steps;                 /* config.train.batch_size (accelerate_ppo_model.py:131) */
} trlx_kl_ctl;

/* state = {mean 0, var 1, std 1, count 1e-24, ref_mean, ref_std, ref_set, init_kl_coef, ...}
 * (RunningMoments.__init__, modeling.py:78-81; orchestrator :48-49; kl_ctl init). */
int trlx_ctl_init(double* state, double init_kl_coef, double ref_mean, double ref_std, int ref_set,
                  void* stream);
/* {Σx, Σx², n, 0} of scores (fp64, one workgroup) — the record a caller all-reduces across
 * ranks before trlx_score_ctl_update / trlx_ppo_rollout_gae_ctl. */
int trlx_score_moments(const void* scores, int dtype, int64_t n, double* moments, void* stream);
/* trlx_score_moments with `done_event` (a hipEvent_t) recorded by the kernel's own dispatch
 * (hipExtLaunchKernel stop event) instead of a separate hipEventRecord marker between this
 * launch and the next: the ordering point the RCCL helper's side stream waits on before the
 * score-moments all-reduce. */
int trlx_score_moments_signal(const void* scores, int dtype, int64_t n, double* moments, void* stream,
                              void* done_event);
/* One workgroup: the score-side control above; scores_out (may alias scores) receives the
 * scaled, clipped scores.  ppo_orchestrator.py:96-112. */
int trlx_score_ctl_update(const void* scores, int dtype, int64_t n, const trlx_score_ctl* ctl,
                          void* scores_out, int out_dtype, void* stream);
/* kl_ctl.update with approx_kl read from device memory (fp32, e.g. the loss stats slot 8). */
int trlx_kl_ctl_update(const trlx_kl_ctl* kl, const float* approx_kl, void* stream);
/* The fused step's tails with the controller state folded in (no extra launch):
 *   trlx_ppo_rollout_gae_ctl  = trlx_ppo_rollout_gae with beta read from ctl->state_in and
 *                               the scores passed through the score-side control (every
 *                               block derives the same values; block 0 writes state_out,
 *                               which must not alias state_in);
 *   trlx_ppo_rollout_loss_ctl = trlx_ppo_rollout_loss + kl_ctl.update(approx_kl) by the
 *                               block that writes the stats. */
int trlx_ppo_rollout_gae_ctl(int64_t B, int64_t T, const float* lp, const float* ref_lp, const void* values,
                             int v_dtype, const float* scores, const int64_t* lengths, const int64_t* mask,
                             const trlx_score_ctl* ctl, float gamma, float lam, float* rewards, float* adv_raw,
                             void* ret, int ret_dtype, double* stats, void* workspace, void* stream);
int trlx_ppo_rollout_loss_ctl(int64_t B, int64_t T, const double* stats, float vf_coef, float* loss,
                              float* loss_stats, void* workspace, const trlx_kl_ctl* kl, void* stream);
/* trlx_lsm_gather_fwd (the next step's experience rows) with the PREVIOUS step's loss tail
 * (trlx_ppo_rollout_loss[_ctl] over tail_B x tail_T token records of `workspace`; kl may be
 * NULL) folded in as the launch's first workgroups: the tail's ~9 us latency-bound
 * reduction and its launch leave the critical path and no cross-stream event is needed.
 * Kernels that cannot host it (the streaming rows) run the tail as its own launch first.
 * Stream order is that of the two calls: the tail reads the token records of the loss rows
 * launched before, the GAE tail launched after reads the KL coefficient it updates.
 * lengths, order_ws: as in trlx_lsm_gather_fwd_ragged (NULL: every row / natural order). */
int trlx_lsm_gather_fwd_loss_tail(const void* x0, const void* x1, int dtype, int64_t B, int64_t T, int64_t V,
                                  int64_t sb, int64_t st, const int64_t* labels, int64_t lb, int64_t lt,
                                  const int64_t* lengths, void* order_ws, void* out_lp0, void* out_lp1, int out_dtype,
                                  int64_t tail_B, int64_t tail_T,
                                  const double* tail_stats, float vf_coef, float* loss, float* loss_stats,
                                  void* workspace, const trlx_kl_ctl* kl, void* stream);

/* ---------------------------------------------------------------- split-beta step (DP pipeline)
 * The KL-penalised reward r = score_t - beta*kl_t (ppo_orchestrator.py:163-167) enters GAE
 * (ppo_models.py:121-139) linearly, so A = A0 - beta*Ak with A0 the GAE of the score +
 * value terms and Ak the discounted KL sums.  Splitting them lets the GAE launch run before
 * the previous batch's KL-controller update (accelerate_ppo_model.py:123,130-131), which the
 * pipelined data-parallel schedule needs to keep its loss tail folded.
 *   trlx_ppo_rollout_gae_split  one wave per rollout: adv0 = A0, adv_kl = Ak, rew_kl = kl_t
 *       (0 past the length), rew_score = the score term (-0.0 before the last column, 0 past
 *       it) and the split record stats8 = {Σ A0, Σ A0², n, Σ Ak, Σ A0·Ak, Σ Ak², Σ mask, 0}
 *       (all-reduce the first 6, or 7 for a global loss normaliser).  ctl: score control as
 *       in trlx_ppo_rollout_gae_ctl (may be NULL); beta is not read.  prev_stats8 (optional):
 *       block 0 also writes the whitening coefficients of the PREVIOUS batch to prev_coef,
 *       with beta = ctl->state_in[TRLX_CTL_KL_COEF] (or kl_coef without ctl).  mom_lag = 1:
 *       ctl->global_moments are the PREVIOUS batch's all-reduced score moments, merged into
 *       RunningMoments now (NULL: none yet); not with TRLX_SCALE_RUNNING.  done_event (a
 *       hipEvent_t or NULL) is recorded by the launch's own dispatch.
 *   trlx_ppo_whiten_coef  the same coefficients as a launch of its own (ctl_state may be NULL):
 *       coef = {mean, rsqrt(var + 1e-8), beta, 0} of A = A0 - beta*Ak (modeling.py:24-34;
 *       unbiased: torch.var_mean, else the distributed biased variance).
 *   trlx_ppo_loss_rows_split  trlx_ppo_loss_rows with the advantage A0 - coef[2]*Ak whitened
 *       by coef, the mask sum at *msum (stats8 + 6), and this batch's rewards
 *       (-beta*rew_kl + rew_score) and returns (A + old_values, r_dtype) written here.  The
 *       loss tail takes stats8 + 3 as its `stats` (it reads Σ mask at stats[3]). */
int trlx_ppo_rollout_gae_split(int64_t B, int64_t T, const float* lp, const float* ref_lp, const void* values,
                               int v_dtype, const float* scores, const int64_t* lengths, const int64_t* mask,
                               const trlx_score_ctl* ctl, float kl_coef, float gamma, float lam, float* adv0,
                               float* adv_kl, float* rew_kl, float* rew_score, double* stats8,
                               const double* prev_stats8, float* prev_coef, int prev_unbiased, int mom_lag,
                               void* workspace, void* stream, void* done_event);
/* RunningMoments merge of an all-reduced {Σx, Σx², n} score record into the controller
 * state (state_out may alias state_in): the last merge of a pipelined sequence whose GAE
 * launches merged each batch's moments one batch late (mom_lag = 1 above: the scores are not
 * scaled by the running std, so the merge can wait for the moments' all-reduce to hide
 * behind the next batch's rows). */
int trlx_score_moments_merge(const double* state_in, double* state_out, const double* moments, void* stream);
int trlx_ppo_whiten_coef(const double* stats8, int unbiased, const double* ctl_state, float kl_coef, float* coef,
                         void* stream);
int trlx_ppo_loss_rows_split(const void* logits, int dtype, int64_t B, int64_t T, int64_t V, int64_t sb,
                             int64_t st, const int64_t* labels, int64_t lb, int64_t lt, const void* old_lp,
                             int old_dtype, const float* adv0, const float* adv_kl, const float* rew_kl,
                             const float* rew_score, const float* coef, const double* msum, const int64_t* mask,
                             const void* values, int v_dtype, const void* old_values, int ov_dtype, float* rewards,
                             void* returns, int r_dtype, float cliprange, float cliprange_value, float vf_coef,
                             float* lp_out, void* dx, int64_t dsb, int64_t dst, float* dvalues, void* workspace,
                             void* stream);
/* The arguments of trlx_ppo_rollout_gae_split (without the previous-batch coefficients and
 * the done event) as one POD, for a GAE folded into another launch. */
typedef struct {
    int64_t B, T;
    const float* lp;
    const float* ref_lp;
    const void* values;
    int v_dtype;
    const float* scores;              /* [B] or NULL */
    const int64_t* lengths;           /* [B] or NULL */
    const int64_t* mask;              /* [B,T] or NULL */
    const trlx_score_ctl* ctl;        /* or NULL */
    float kl_coef, gamma, lam;
    float* adv0;
    float* adv_kl;
    float* rew_kl;
    float* rew_score;
    double* stats8;
    int mom_lag;
    void* workspace;                  /* trlx_ppo_workspace_bytes(B, T) */
} trlx_gae_split_args;
/* trlx_ppo_loss_rows_split of batch k whose rows derive the whitening coefficients
 * themselves — coef = {mean, rsqrt(var + 1e-8), beta, 0} of A = A0 - beta*Ak from the
 * (all-reduced) split record stats8, beta = ctl_state[TRLX_CTL_KL_COEF] or kl_coef when
 * ctl_state is NULL (modeling.py:24-34) — so no coefficient launch sits between the record's
 * all-reduce and the rows; row 0 stores them to `coef` for a later trlx_ppo_loss_rows_split on
 * the same experience (the ppo_epochs pattern: beta stays the experience's).  `gae` (or NULL):
 * the split GAE of the NEXT batch (ppo_orchestrator.py:163-167, ppo_models.py:121-139) runs as
 * this launch's first workgroups — nothing in it depends on these rows, so the pipelined DP
 * schedule needs no GAE launch of its own.  It must write the other split buffer set; with a
 * ctl it reads ctl->state_in and writes ctl->state_out, and ctl_state here must not be the
 * state_out.  done_event (a hipEvent_t or NULL) is recorded by the launch's own dispatch. */
int trlx_ppo_loss_rows_split_gae(const void* logits, int dtype, int64_t B, int64_t T, int64_t V, int64_t sb,
                                 int64_t st, const int64_t* labels, int64_t lb, int64_t lt, const void* old_lp,
                                 int old_dtype, const float* adv0, const float* adv_kl, const float* rew_kl,
                                 const float* rew_score, const double* stats8, int unbiased, const double* ctl_state,
                                 float kl_coef, float* coef, const double* msum, const int64_t* mask,
                                 const void* values, int v_dtype, const void* old_values, int ov_dtype,
                                 float* rewards, void* returns, int r_dtype, float cliprange, float cliprange_value,
                                 float vf_coef, float* lp_out, void* dx, int64_t dsb, int64_t dst, float* dvalues,
                                 void* workspace, const trlx_gae_split_args* gae, void* stream, void* done_event);

/* ---------------------------------------------------------------- RCCL stats all-reduce helper
 * SURVEY §8b "Collectives" — replaces the two dist.all_reduce calls of
 * get_global_statistics (trlx/utils/modeling.py:13-14, 18-19) on the hot path: ONE
 * communicator per process, SUM of a small fp64 vector ({Σx, Σx², n[, Σmask]} or the score
 * moments) enqueued on the caller's HIP stream — no side stream, no system-scope event join
 * (each of ProcessGroupNCCL's costs ~20 us of compute-queue idle on MI355X).
 *   trlx_comm_load      dlopen the RCCL the process already uses (PyTorch's librccl.so path)
 *   trlx_comm_unique_id rank 0: ncclGetUniqueId into a trlx_comm_unique_id_bytes() buffer,
 *                       which the caller broadcasts (the bindings use torch.distributed)
 *   trlx_comm_init      every rank, collectively: ncclCommInitRank on the current HIP device
 *   trlx_comm_allreduce_sum_f64   in-place SUM of buf[0:n] on `stream`
 *   trlx_comm_destroy   ncclCommDestroy */
int trlx_comm_load(const char* librccl_path);
int64_t trlx_comm_unique_id_bytes(void);
int trlx_comm_unique_id(void* id_out, int64_t nbytes);
int trlx_comm_init(void** comm_out, const void* id, int64_t nbytes, int nranks, int rank);
int trlx_comm_allreduce_sum_f64(void* comm, double* buf, int64_t n, void* stream);
int trlx_comm_destroy(void* comm);

/* ---------------------------------------------------------------- autograd plumbing
 * out[i] = x[i] * (*scale) for i < n (scale: device fp32 scalar, e.g. a backward's
 * grad_output).  In place (out == x) it is skipped entirely when *scale == 1. */
int trlx_scale_by(const void* x, void* out, int dtype, int64_t n, const float* scale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TRLX_T5_AMD_H */
