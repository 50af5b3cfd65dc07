/*
 * twotower_amd.h — C ABI of the MI355X (gfx950) two-tower training-step library
 * (libtwotower_amd.so).
 *
 * Every entry point replaces one device op that the reference (k0r1g/two-towers, pure
 * PyTorch) reaches through ATen on its hot path.  The reference has no FFI of its own;
 * the Python host package `twotower_amd` binds these symbols with ctypes behind the
 * reference's plugin surface (BaseEmbedding / BaseTower / LOSS_REGISTRY).  Each
 * declaration cites the reference call site it replaces.
 *
 * Conventions
 *   - All pointers are DEVICE pointers owned by the caller (PyTorch's caching allocator).
 *     The library never allocates; scratch comes in through `ws`/`ws_bytes`.
 *   - `stream` is the caller's hipStream_t (the torch current stream); every launch is
 *     asynchronous on it, nothing synchronises, so calls are graph-capturable.
 *   - Return value: 0 = success; > 0 = hipError_t of a failed launch; < 0 = TT_ERR_*
 *     argument validation failure.  tt_last_error() returns the thread's last message.
 *   - fp32 matrices are row-major, contiguous (leading dimension = row length) unless a
 *     leading-dimension argument says otherwise.
 */
#ifndef TWOTOWER_AMD_H
#define TWOTOWER_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* tt_stream_t; /* layout-compatible with hipStream_t */

enum tt_status { TT_OK = 0, TT_ERR_INVALID = -1, TT_ERR_WORKSPACE = -2, TT_ERR_UNSUPPORTED = -3 };
enum tt_index_dtype { TT_IDS_I32 = 0, TT_IDS_I64 = 1 };
enum tt_compute_dtype { TT_F32 = 0, TT_BF16 = 1, TT_BF16_SPLIT = 2 };
enum tt_scatter_mode {
  TT_SCATTER_SORTED = 0, /* deterministic: stable radix sort + segmented row reduce; writes every row */
  TT_SCATTER_ATOMIC = 1  /* global_atomic_add_f32 into caller-zeroed grad; order-dependent */
};

/* ---- library ------------------------------------------------------------------ */
int tt_version(void);
const char* tt_last_error(void);

/* ---- embedding bag: lookup + masked mean-pool -----------------------------------
 * Replaces, per tower call:
 *   LookupEmbedding.forward  -> nn.Embedding(V,E,padding_idx=0)(ids)   twotower/embeddings.py:30,40
 *   MeanPoolingTower.forward  mask=(ids>0) :62, emb*mask :67, sum(1)/(mask.sum(1)+1e-9) :72
 *                                                                    twotower/encoders.py:62-72
 * pooled[s,:] = sum_{t: ids[s,t]>0} table[ids[s,t],:] / denom[s],  denom[s] = count + 1e-9f.
 * ids are (nseq, L) with row stride ld_ids elements, int32 or int64 (the reference feeds int64,
 * twotower/dataset.py:274-278).  Ids >= V are treated as masked (the reference raises). */
int tt_bag_mean_fwd(const float* table, int64_t V, int E,
                    const void* ids, int ids_dtype, int64_t nseq, int L, int64_t ld_ids,
                    float* pooled, float* denom, tt_stream_t stream);
/* tt_bag_mean_fwd over a column slab (table_sync "column": this rank's El columns of every row,
 * slab V x El): pooled (nseq x El) summed in the order tt_bag_mean_fwd sums those columns at the
 * full width E, so the assembled rows equal the one-GPU forward's bit for bit.  El in
 * {32, 64, 128, 256} dividing E.  Replaces the reference's per-rank embedding lookup + masked mean
 * (twotower/embeddings.py:30, encoders.py:67-72) for a column-sharded table. */
int tt_bag_mean_fwd_cols(const float* slab, int64_t V, int El, int E,
                         const void* ids, int ids_dtype, int64_t nseq, int L, int64_t ld_ids,
                         float* pooled, float* denom, tt_stream_t stream);
/* tt_bag_mean_fwd whose launch also forms the four weight plane sets of the tower head that
 * consumes the pooled rows (W1 H x E, W2 H x H: tt_head_split_ff2's output in `planes`, bit for
 * bit) in extra workgroups, so the split leaves the path between the gather and the first head
 * GEMM (MeanPoolingTower, encoders.py:38-42).  E in {64, 128, 256}, H in {128, 256}. */
int tt_bag_mean_fwd_split(const float* table, int64_t V, int E,
                          const void* ids, int ids_dtype, int64_t nseq, int L, int64_t ld_ids,
                          float* pooled, float* denom, const float* W1, const float* W2, int H,
                          void* planes, tt_stream_t stream);

/* Backward of the above w.r.t. the table (autograd of encoders.py:67-72 +
 * embedding_dense_backward with padding_idx, reached from twotower/train.py:138):
 *   G[id,:] += d_pooled[s,:] / denom[s] for every token with 0 < id < V, id != padding_idx.
 * TT_SCATTER_SORTED overwrites all V rows of grad_table (untouched rows -> 0);
 * TT_SCATTER_ATOMIC accumulates into grad_table (caller zeroes it; ws may be NULL). */
size_t tt_bag_mean_bwd_ws_size(int64_t nseq, int L, int64_t V, int E);
int tt_bag_mean_bwd(const float* d_pooled, const float* denom,
                    const void* ids, int ids_dtype, int64_t nseq, int L, int64_t ld_ids,
                    int64_t V, int E, int64_t padding_idx, float* grad_table, int mode,
                    void* ws, size_t ws_bytes, tt_stream_t stream);

/* Sorted scatter fused with a dense AdamW step on the table (exactly the math of
 * tt_bag_mean_bwd(SORTED) followed by tt_adamw on the table, without materialising G):
 * replaces embedding_dense_backward + torch.optim.AdamW.step for the table,
 * twotower/train.py:138-139,359.  Every row is updated (rows without tokens see g = 0). */
int tt_bag_mean_bwd_adamw(const float* d_pooled, const float* denom,
                          const void* ids, int ids_dtype, int64_t nseq, int L, int64_t ld_ids,
                          int64_t V, int E, int64_t padding_idx,
                          float* table, float* exp_avg, float* exp_avg_sq,
                          double lr, double beta1, double beta2, double eps, double weight_decay,
                          int64_t step, void* ws, size_t ws_bytes, tt_stream_t stream);

/* Split form of the sorted backward, so the id-only half can run early (beside the forward, on
 * another stream) and a step can be captured in a HIP graph:
 *   tt_bag_plan         ids -> sorted (row, seq) pairs + per-row segment bounds, into `plan`
 *                       (tt_bag_plan_ws_size bytes; it also holds the scaled-row scratch);
 *   tt_bag_mean_bwd_planned        dense grad_table from d_pooled/denom and the plan;
 *   tt_bag_mean_bwd_adamw_planned  fused AdamW with the per-step scalars read from device
 *                       memory (`adam_args`, written by tt_adam_prepare).
 * Plan + apply compute exactly what tt_bag_mean_bwd / tt_bag_mean_bwd_adamw compute.  In the two
 * apply calls denom may be NULL: d_pooled then already holds gs = d_pooled / denom (formed by
 * the tower head's dx epilogue, tt_head_gemm epi 5) and the scaling pass is skipped. */
size_t tt_bag_plan_ws_size(int64_t nseq, int L, int64_t V, int E);
int tt_bag_plan(const void* ids, int ids_dtype, int64_t nseq, int L, int64_t ld_ids,
                int64_t V, int E, int64_t padding_idx, void* plan, size_t plan_bytes,
                tt_stream_t stream);
int tt_bag_mean_bwd_planned(const float* d_pooled, const float* denom, int64_t nseq, int L,
                            int64_t V, int E, const void* plan, size_t plan_bytes,
                            float* grad_table, tt_stream_t stream);
/* Where the plan's sorted output lies inside `plan` (byte offsets from the plan pointer rounded
 * up to 256 B): offs[0] the sorted row keys (room for nseq*L uint32), offs[1] their sequence
 * indices (room for nseq*L int32), offs[2] seg_start (V + 1 int32: row r's entries are
 * [seg_start[r], seg_start[r + 1])).  The sort is the stable sort of the kept (row, seq) pairs by
 * row, so these are fixed by the ids: what the parity tests compare with a CPU stable sort.  The
 * masked slots (pads, padding_idx, ids outside (0, V)) are dropped: seg_start[V] entries are
 * written, the rest of the two arrays is unspecified. */
int tt_bag_plan_layout(int64_t nseq, int L, int64_t V, int E, int64_t* offs);
/* tt_bag_plan in two halves on one stream (same plan, same bytes): part 0 runs every sort pass
 * but the last, part 1 the last pass, the segment starts and the pieces, so a caller can place the
 * second half later in its step (the same ids and plan buffer in both calls). */
int tt_bag_plan_part(const void* ids, int ids_dtype, int64_t nseq, int L, int64_t ld_ids,
                     int64_t V, int E, int64_t padding_idx, void* plan, size_t plan_bytes, int part,
                     tt_stream_t stream);
int tt_bag_mean_bwd_adamw_planned(const float* d_pooled, const float* denom, int64_t nseq, int L,
                                  int64_t V, int E, const void* plan, size_t plan_bytes,
                                  float* table, float* exp_avg, float* exp_avg_sq,
                                  const void* adam_args, tt_stream_t stream);

/* Row-range form of tt_bag_mean_bwd_planned, for a data-parallel table gradient exchanged in
 * row chunks (the row-sharded optimizer pipelines each chunk's reduce-scatter / AdamW /
 * all-gather behind the next chunk's gradient; the exchange sits where the reference runs
 * loss.backward(); optimizer.step(), twotower/train.py:138-139):
 *   tt_bag_mean_bwd_planned_prepare  once per step: gs = d_pooled / denom (skipped when denom is
 *                       NULL) and the long rows' piece sums, into the plan workspace;
 *   tt_bag_mean_bwd_planned_rows     rows [row_begin, row_end) of the dense gradient into
 *                       grad_rows ((row_end - row_begin) x E), the same sums in the same order as
 *                       tt_bag_mean_bwd_planned writes for those rows. */
int tt_bag_mean_bwd_planned_prepare(const float* d_pooled, const float* denom, int64_t nseq, int L,
                                    int64_t V, int E, void* plan, size_t plan_bytes,
                                    tt_stream_t stream);
int tt_bag_mean_bwd_planned_rows(const float* d_pooled, const float* denom, int64_t nseq, int L,
                                 int64_t V, int E, const void* plan, size_t plan_bytes,
                                 int64_t row_begin, int64_t row_end, float* grad_rows,
                                 tt_stream_t stream);
/* tt_bag_mean_bwd_adamw_planned_rows: rows [row_begin, row_end) of tt_bag_mean_bwd_adamw_planned
 *   (after tt_bag_mean_bwd_planned_prepare on the same stream): the same sums in the same order,
 *   then AdamW on those rows, whose parameters and moments are table_rows / exp_avg_rows /
 *   exp_avg_sq_rows ((row_end - row_begin) x E each).  The data-parallel "owner" table exchange
 *   (optim.AdamW): the plan covers every rank's tokens (all-gathered ids, d_pooled / denom), and each
 *   rank updates only the rows it owns, with its shard of the moments, before the rows are
 *   all-gathered (twotower/train.py:138-139). */
int tt_bag_mean_bwd_adamw_planned_rows(const float* d_pooled, const float* denom, int64_t nseq, int L,
                                       int64_t V, int E, const void* plan, size_t plan_bytes,
                                       int64_t row_begin, int64_t row_end, float* table_rows,
                                       float* exp_avg_rows, float* exp_avg_sq_rows, const void* adam_args,
                                       tt_stream_t stream);

/* ---- column-sharded table (data parallel, optim.AdamW(table_sync="column")) -------------------
 * Replaces, per rank, the embedding's dense backward + AdamW (twotower/embeddings.py:30 via
 * train.py:138-139) for the columns [c0, c0 + El) this rank owns of every table row (its slab,
 * V x El, and the slab's moments).  The forward is tt_bag_mean_fwd over the slab with every rank's
 * ids (E = El); these two entry points are the backward:
 *   tt_bag_scale_rows  gs = d_pooled / denom per row (the division autograd applies at
 *                      encoders.py:72), nseq x E, before gs is exchanged all-to-all by columns;
 *   tt_bag_col_reduce  row r's gradient = the sum of gs over every rank's tokens of row r, from the
 *                      all-gathered per-rank plans (tt_bag_plan): seg_all (nsrc x (V + 1)) row
 *                      starts and vals_all (nsrc x nL) sorted sequence indices of source src's
 *                      nseq sequences, gs_all (nsrc * nseq x El) row src * nseq + s.  The sources
 *                      are merged in rank order inside the reduce (the global batch's stable order),
 *                      with tt_bag_mean_bwd_planned's interleaved partial sums.  grad != NULL: the
 *                      gradient rows (V x El) are written; grad == NULL: AdamW on slab / exp_avg /
 *                      exp_avg_sq with the device scalars adam_args (tt_adam_prepare).
 *                      El in {32, 64, 128, 256}. */
int tt_bag_scale_rows(const float* d_pooled, const float* denom, int64_t nseq, int E, float* gs,
                      tt_stream_t stream);
int tt_bag_col_reduce(const int32_t* seg_all, const int32_t* vals_all, int64_t nL, int nsrc, int64_t nseq,
                      const float* gs_all, int64_t V, int El, float* grad, float* slab, float* exp_avg,
                      float* exp_avg_sq, const void* adam_args, tt_stream_t stream);
/* tt_bag_col_reduce with the hot-row path (embeddings.py:30 under Zipf ids; the 33-row character
 * vocabulary of tokenisers.py:50,59): with a workspace of tt_bag_col_reduce_ws_size bytes, a row whose
 * merged length exceeds 128 tokens is summed in pieces first (one sub-wave per piece, in the merged
 * order), then folded -- the single-plan path's pieces and folds for rows of up to 32,768 merged tokens
 * (bit for bit equal to tt_bag_mean_bwd(_adamw)_planned over the concatenated batch), up to 4,096
 * pieces and a group level beyond.  ws == NULL: tt_bag_col_reduce (every row walked by one sub-wave). */
size_t tt_bag_col_reduce_ws_size(int64_t V, int nsrc, int64_t nL, int El);
int tt_bag_col_reduce_ex(const int32_t* seg_all, const int32_t* vals_all, int64_t nL, int nsrc, int64_t nseq,
                         const float* gs_all, int64_t V, int El, float* grad, float* slab, float* exp_avg,
                         float* exp_avg_sq, const void* adam_args, void* ws, size_t ws_bytes, tt_stream_t stream);

/* ---- dense AdamW (torch.optim.AdamW, twotower/train.py:359, .step() :139) ---------
 * p *= 1 - lr*wd;  m = lerp(m, g, 1-b1);  v = b2*v + (1-b2)*g*g;
 * p -= lr/(1-b1^step) * m / (sqrt(v)/sqrt(1-b2^step) + eps).   step is 1-based.
 * Hyper-parameters are double: like torch, the per-step scalars (1-b2, bias corrections) are
 * formed in double and rounded to float once (1 - (float)0.999 would be off by 1.3e-5). */
int tt_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
             double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step,
             tt_stream_t stream);

/* Device-resident form (graph-capturable; torch's capturable=True convention of a device `step`):
 * tt_adam_prepare increments each slot's fp32 step counter on the device and writes that
 * tensor's per-step scalars (same double-precision formulas as above) into `args`
 * (TT_ADAM_ARGS_BYTES device bytes, 4-byte aligned); tt_adamw_multi then updates up to
 * TT_ADAM_MAX_TENSORS tensors in one launch, each with its own args. */
#define TT_ADAM_ARGS_BYTES 32
#define TT_ADAM_MAX_TENSORS 16
#define TT_ADAM_TICKET_WORDS 16 /* tt_adamw_multi_ex's ticket: zeroed device words (it uses 9) */
typedef struct {
  float* step;
  void* args;
} tt_adam_slot;
typedef struct {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t n;
  const void* args;
} tt_adamw_tensor;
int tt_adam_prepare(const tt_adam_slot* slots, int count, double lr, double beta1, double beta2,
                    double eps, double weight_decay, tt_stream_t stream);
/* tt_adam_prepare_ex: step += increment (0 or 1), then the scalars of step + ahead (0 or 1).
 * tt_adam_prepare is (1, 0).  (1, 1) after a step's updates forms the NEXT step's scalars while
 * advancing the counter, so that step's updates need no prepare launch in front of them;
 * (0, 1) forms them for counters nobody prepared ahead (first step, new hyper-parameters). */
int tt_adam_prepare_ex(const tt_adam_slot* slots, int count, double lr, double beta1, double beta2,
                       double eps, double weight_decay, int increment, int ahead, tt_stream_t stream);
int tt_adamw_multi(const tt_adamw_tensor* tensors, int count, tt_stream_t stream);
/* tt_adamw_multi_ex: tt_adamw_multi that can also (1) form a tensor's gradient from slab
 * partials first -- parts[i].part != NULL: grad[k] = the fixed-order slab sum of
 * part[s * stride + k], s < slabs, the same sum tt_head_wgrad2_reduce forms, written to
 * tensors[i].grad (which must then be writable, 16-byte aligned, n % 4 == 0) and used -- and
 * (2) run tt_adam_prepare_ex(next, nnext, ..., increment 1, ahead 1) in the same launch, after
 * every update has read its scalars (the last workgroup to finish, by a ticket: `ticket` is
 * TT_ADAM_TICKET_WORDS zeroed device unsigneds the kernel leaves zeroed).  parts may be NULL;
 * nnext 0 skips (2).
 * The tail of a step as one launch instead of slab sums + updates + prepare. */
typedef struct {
  const float* part;
  int64_t stride;  /* floats between slabs */
  int slabs;
} tt_adamw_grad_parts;
int tt_adamw_multi_ex(const tt_adamw_tensor* tensors, const tt_adamw_grad_parts* parts, int count,
                      const tt_adam_slot* next, int nnext, double lr, double beta1, double beta2, double eps,
                      double weight_decay, unsigned* ticket, tt_stream_t stream);

/* ---- mean of n floats (the loss reductions' F.cross_entropy / .mean(), losses.py:44,85,116):
 * one workgroup, fixed-order sums (bitwise reproducible); the in-batch forward forms it itself
 * unless its loss pointer is NULL. */
int tt_mean(const float* x, int64_t n, float* out, tt_stream_t stream);

/* ---- row L2 normalise (F.normalize(x, dim=-1), eps 1e-12; twotower/encoders.py:77) -- */
int tt_l2norm_fwd(const float* x, int64_t rows, int H, float* out, float* norm, tt_stream_t stream);
int tt_l2norm_bwd(const float* dout, const float* out, const float* norm, int64_t rows, int H,
                  float* dx, tt_stream_t stream);

/* ---- LayerNorm + L2 normalise (AveragePoolingTower projection tail: nn.LayerNorm(H) then
 * F.normalize, twotower/encoders.py:95-97,150).  fwd: out and per-row stats (mean, rstd, |y|,
 * 3 floats per row).  bwd: dx, and the per-row gamma / beta gradient terms gx = dy*xhat, gb = dy
 * (rows x H each; their column sums are dgamma / dbeta, tt_colsum). */
int tt_ln_l2_fwd(const float* x, int64_t rows, int H, const float* gamma, const float* beta, float eps, float* out,
                 float* stats, tt_stream_t stream);
int tt_ln_l2_bwd(const float* dout, const float* x, int64_t rows, int H, const float* gamma, const float* beta,
                 const float* stats, float* dx, float* gx, float* gb, tt_stream_t stream);
/* tt_ln_l2_bwd_ex: dx and the gamma / beta gradients themselves (the per-row terms folded over
 * each workgroup's rows, then column-summed; fixed order), with a workspace of
 * tt_ln_l2_bwd_ws_size bytes; H even, <= 1024. */
size_t tt_ln_l2_bwd_ws_size(int64_t rows, int H);
int tt_ln_l2_bwd_ex(const float* dout, const float* x, int64_t rows, int H, const float* gamma, const float* beta,
                    const float* stats, float* dx, float* dgamma, float* dbeta, void* ws, size_t ws_bytes,
                    tt_stream_t stream);

/* ---- column sum (bias gradient of nn.Linear: grad_out.sum(0); twotower/encoders.py:38-42) ----
 * out[c] = sum_r x[r, c] in a fixed order (deterministic): per-block partial sums over row
 * chunks into ws (>= tt_colsum_ws_size bytes), then one fixed-order pass over the partials. */
size_t tt_colsum_ws_size(int64_t rows, int cols);
int tt_colsum(const float* x, int64_t rows, int cols, float* out, void* ws, size_t ws_bytes, tt_stream_t stream);

/* ---- ReLU backward in place (nn.ReLU between the tower Linears, encoders.py:40):
 * dh[i] = h[i] > 0 ? dh[i] : 0 (16-byte vectors when n % 4 == 0 and both are aligned). */
int tt_relu_bwd(float* dh, const float* h, int64_t n, tt_stream_t stream);

/* ---- triplet hinge on cosine (contrastive_triplet_loss, twotower/losses.py:9-44) ----
 * loss = mean_i relu(margin - cos(q_i,p_i) + cos(q_i,n_i)), cosine eps 1e-8.
 * fwd writes loss_rows[B] and loss[1]; bwd reads the upstream scalar grad from grad_loss
 * (device) and writes dq, dp, dn. */
int tt_triplet_fwd(const float* q, const float* p, const float* n, int64_t B, int H,
                   float margin, float* loss_rows, float* loss, tt_stream_t stream);
int tt_triplet_bwd(const float* q, const float* p, const float* n, int64_t B, int H,
                   float margin, const float* grad_loss, float* dq, float* dp, float* dn,
                   tt_stream_t stream);

/* ---- InfoNCE with N negatives (multiple_negatives_loss, twotower/losses.py:47-85) ----
 * logits[i,k] = cos(q_i, [p_i, negs_i,0..N-1][k]) / tau; loss = mean_i CE(logits_i, 0). */
int tt_multi_neg_fwd(const float* q, const float* p, const float* negs, int64_t B, int N, int H,
                     float inv_tau, float* loss_rows, float* loss, tt_stream_t stream);
int tt_multi_neg_bwd(const float* q, const float* p, const float* negs, int64_t B, int N, int H,
                     float inv_tau, const float* grad_loss, float* dq, float* dp, float* dnegs,
                     tt_stream_t stream);
/* tt_multi_neg_bwd fused with the tower head's F.normalize backward (encoders.py:77), H = 256,
 * N <= 15: qpn is the head's output [q; p; negs] ((2 + N) B x 256, the normalised rows), norms its
 * row norms in the same order; dx (same shape) receives the gradient before F.normalize, equal bit
 * for bit to tt_multi_neg_bwd followed by tt_l2norm_bwd on those rows. */
int tt_multi_neg_bwd_l2(const float* qpn, int64_t B, int N, const float* norms, float inv_tau,
                        const float* grad_loss, float* dx, tt_stream_t stream);

/* ---- in-batch sampled softmax (in_batch_sampled_softmax_loss, twotower/losses.py:88-118)
 * S = q d^T (B x M, never materialised), logits = S * inv_tau, label of row i is column
 * i + label_off (reference: arange(B), label_off = 0; data-parallel: rank * local M).
 * loss = mean_i (lse_i - logits[i, i+label_off]).
 * compute dtype TT_F32 (exact fp32 MFMA), TT_BF16 (bf16 MFMA operands, P rounded once to bf16,
 * fp32 accumulation) or TT_BF16_SPLIT (P split hi + lo bf16 so the P.D / dS^T.Q products keep
 * ~16 mantissa bits, at 1.5x the MFMA work; the q/d rounding to bf16 still dominates the error
 * against fp32 inputs: both bf16 forms land ~3-4e-3 from the fp32 reference's gradients at C3).
 * fwd (want_grad != 0) also leaves dq_unscaled = sum_j P_ij d~_j - d~_label (B x H) so the
 * backward needs only the dD pass.  ws must stay untouched between fwd and bwd: it carries the
 * bf16 operands, the pad rows and lse in log2 units, which the backward engine reads (the lse
 * argument of tt_inbatch_bwd is the same quantity, validated but not re-read).  In the default
 * backward form (TT_INBATCH_BWD_STORED) the TT_BF16 workspace also carries the forward's bf16
 * probabilities (about B * M * 2 bytes, kept while B * M <= 2^31) and a rescaled bf16 copy of q,
 * from which the backward forms P without recomputing S; the TT_F32 workspace likewise carries
 * fp32 probabilities (about B * M * 4 bytes, kept while B * M <= 2^30) and a rescaled fp32 copy
 * of q (TT_BF16_SPLIT always recomputes).
 * tt_inbatch_set_backward(mode) selects the form process-wide and returns the previous one (an
 * unknown mode only reads it); the initial form is STORED unless the environment sets
 * TT_INBATCH_BWD=recompute.  The workspace size depends on the form: size it after selecting, and
 * do not switch between a forward and its backward. */
#define TT_INBATCH_BWD_RECOMPUTE 0
#define TT_INBATCH_BWD_STORED 1
int tt_inbatch_set_backward(int mode);
size_t tt_inbatch_ws_size(int64_t B, int64_t M, int H, int dtype);
int tt_inbatch_fwd(const float* q, const float* d, int64_t B, int64_t M, int H, int dtype,
                   float inv_tau, int64_t label_off, int want_grad,
                   float* lse, float* loss_rows, float* loss, float* dq_unscaled,
                   void* ws, size_t ws_bytes, tt_stream_t stream);
/* dq = grad_loss[0]*grad_scale*inv_tau*dq_unscaled;
 * dd[j] = grad_loss[0]*grad_scale*inv_tau * sum_i (P_ij - [j == i+label_off]) q~_i.
 * grad_scale is 1/B for the reference's mean reduction.
 * loss_rows, loss: both NULL, or the forward's per-row losses (B floats) and where to put their
 * mean, formed in one extra workgroup of the combine launch with tt_mean's arithmetic (the same
 * bits): for a caller whose forward passed loss = NULL because the loss is read only after the
 * backward (train_step.TrainStep), so the mean's own launch leaves the forward-to-backward path. */
int tt_inbatch_bwd(const float* q, const float* d, int64_t B, int64_t M, int H, int dtype,
                   float inv_tau, int64_t label_off, const float* lse, const float* dq_unscaled,
                   const float* grad_loss, float grad_scale, float* dq, float* dd,
                   const float* loss_rows, float* loss, void* ws, size_t ws_bytes, tt_stream_t stream);

/* ---- the same loss from explicit, prepared operands (bf16 / bf16_split only), for data
 * parallelism with candidate-owner gradients (cross-device negatives without a gradient
 * reduce-scatter): each rank prepares its queries and candidates, the caller all-gathers the
 * candidate copies and norm maxima (forward) and the query copies and lse2 (backward), and the
 * backward computes dd for the rank's OWN candidates over every rank's queries.  Replaces the
 * reference's single-device torch.matmul + F.cross_entropy (twotower/losses.py:107-116) when
 * the batch is split over ranks.
 * tt_inbatch_prep_rows: xb (optional) = bf16 copy of x with TT_INBATCH_TAIL_ROWS zero rows after
 *   the last row ((rows + 64) x H storage); norms (optional, rows) = fp32 row L2 norms;
 *   max_parts (optional, TT_INBATCH_MAX_PARTS floats) = per-block max norms, unused entries 0.
 * tt_inbatch_fwd_ex: Qb (B rows) and qnorm of this rank's queries; Db_all (M_all rows + zero
 *   tail) every rank's candidates; dmax_parts (n_parts) every rank's max_parts; labels i +
 *   label_off.  Writes lse, lse2 (log2 units), loss_rows, loss (mean over B), dq_unscaled.
 * tt_inbatch_bwd_ex: Qb_all (nQ_all rows + zero tail) and lse2_all (nQ_all + 64 floats, the
 *   tail +inf) of every rank's queries; Db (M rows) this rank's candidates; the label of
 *   candidate j (0 <= j - label_off < B) is query row q_row0 + j - label_off of Qb_all.
 *   dd[j] = scale sum_i (P_ij - [label]) q~_i over all nQ_all queries, scale =
 *   grad_loss[0] * grad_scale * inv_tau (every rank's loss seeded alike); dq = scale * dq_unscaled.
 * ws: tt_inbatch_ex_ws_size(B, M_all, nQ_all, M) bytes serve both passes (partials only). */
/* tt_inbatch_l2_prep: F.normalize (encoders.py:77) of the B + M rows of y = [q; d] in place, as
 *   tt_head_gemm epi 1 does it (norms[r] = |row|; y the epi 4 output), fused with the operand prep
 *   of tt_inbatch_fwd on the normalised rows, which it leaves in ws (H = 256 with dtype TT_BF16 or
 *   TT_BF16_SPLIT, H = 128 with TT_F32; ws sized by tt_inbatch_ws_size(B, M, H, dtype)).
 * tt_inbatch_fwd_prepped: tt_inbatch_fwd on q = y[:B], d = y[B:] with that workspace, without its
 *   prep pass (bit-identical results). */
int tt_inbatch_l2_prep(float* y, int64_t B, int64_t M, int H, int dtype, float* norms, void* ws, size_t ws_bytes,
                       tt_stream_t stream);
int tt_inbatch_fwd_prepped(const float* q, const float* d, int64_t B, int64_t M, int H, int dtype,
                           float inv_tau, int64_t label_off, int want_grad,
                           float* lse, float* loss_rows, float* loss, float* dq_unscaled,
                           void* ws, size_t ws_bytes, tt_stream_t stream);
/* tt_inbatch_bwd fused with the tower head's F.normalize backward (encoders.py:77), for the fused
 *   TwoTower output qd = [q; d] ((B + M) x H fp32, the rows tt_inbatch_l2_prep normalised,
 *   norms[r] = their norms before it; H = 256 with bf16 / bf16_split operands in ws from the
 *   forward, or H = 128 with fp32 operands): dx ((B + M) x H) = the gradient w.r.t. the rows
 *   before F.normalize, i.e. tt_inbatch_bwd's dq, dd followed by tt_l2norm_bwd, bit for bit,
 *   without writing dq and dd.  loss_rows, loss: as tt_inbatch_bwd (the deferred loss mean). */
int tt_inbatch_bwd_l2(const float* qd, int64_t B, int64_t M, int H, int dtype, float inv_tau, int64_t label_off,
                      const float* lse, const float* dq_unscaled, const float* grad_loss, float grad_scale,
                      const float* norms, float* dx, const float* loss_rows, float* loss, void* ws,
                      size_t ws_bytes, tt_stream_t stream);
#define TT_INBATCH_TAIL_ROWS 64
#define TT_INBATCH_MAX_PARTS 512
int tt_inbatch_prep_rows(const float* x, int64_t rows, int H, void* xb, float* norms, float* max_parts,
                         tt_stream_t stream);
size_t tt_inbatch_ex_ws_size(int64_t B, int64_t M_all, int64_t nQ_all, int64_t M, int H, int dtype);
int tt_inbatch_fwd_ex(const void* Qb, const float* qnorm, int64_t B, const void* Db_all,
                      const float* dmax_parts, int n_parts, int64_t M_all, int H, int dtype, float inv_tau,
                      int64_t label_off, int want_grad, float* lse, float* lse2, float* loss_rows,
                      float* loss, float* dq_unscaled, void* ws, size_t ws_bytes, tt_stream_t stream);
/* The same forward in two launches, so the caller's candidate all-gather overlaps the scoring of
 * the rank's own candidates (bf16 / bf16_split; M and own_begin multiples of 64):
 * tt_inbatch_fwd_ex_local: Db_loc = this rank's candidates (M rows + zero tail), dmax_loc its
 *   n_loc max_parts; scores them with their own norm bound (no other rank's data needed).
 * tt_inbatch_fwd_ex_remote: Db_all, dmax_parts as in tt_inbatch_fwd_ex (own block at rows
 *   [own_begin, own_begin + M), labels i + own_begin); scores the other rows, then combines both
 *   launches (the local partials rescaled to the global bound).  Same outputs as
 *   tt_inbatch_fwd_ex within fp32 rounding; ws sized by tt_inbatch_ex_ws_size(B, M_all, nQ_all, M). */
int tt_inbatch_fwd_ex_local(const void* Qb, const float* qnorm, int64_t B, const void* Db_loc,
                            const float* dmax_loc, int n_loc, int64_t M, int64_t M_all, int64_t own_begin,
                            int H, int dtype, float inv_tau, void* ws, size_t ws_bytes, tt_stream_t stream);
int tt_inbatch_fwd_ex_remote(const void* Qb, const float* qnorm, int64_t B, const void* Db_all,
                             const float* dmax_parts, int n_parts, const float* dmax_loc, int n_loc,
                             int64_t M, int64_t M_all, int64_t own_begin, int H, int dtype, float inv_tau,
                             int want_grad, float* lse, float* lse2, float* loss_rows, float* loss,
                             float* dq_unscaled, void* ws, size_t ws_bytes, tt_stream_t stream);
int tt_inbatch_bwd_ex(const void* Qb_all, const float* lse2_all, int64_t nQ_all, int64_t q_row0,
                      const void* Db, int64_t M, int64_t B, int64_t label_off, int H, int dtype,
                      float inv_tau, const float* dq_unscaled, const float* grad_loss, float grad_scale,
                      float* dq, float* dd, void* ws, size_t ws_bytes, tt_stream_t stream);

/* ---- search over indexed documents (inference/search/two_tower.py:72-115, evaluate.py:159-199)
 * tt_cosine_scores: scores[i*nd + j] = F.cosine_similarity(q_i, d_j) with eps 1e-8 (each side
 *   divided by max(|x|, eps), then summed products); q (nq x H), docs (nd x H) fp32, H % 4 == 0.
 * tt_topk_rows: per row of a (nrows x ncols) score matrix the k largest values, descending, and
 *   their column indices (torch.topk; ties broken by the lower index), 1 <= k <= min(1024, ncols). */
int tt_cosine_scores(const float* q, int64_t nq, const float* docs, int64_t nd, int H, float* scores,
                     tt_stream_t stream);
int tt_topk_rows(const float* scores, int64_t nrows, int64_t ncols, int k, float* out_vals, int64_t* out_idx,
                 tt_stream_t stream);
/* tt_topk_rows_ex: the same result; with a workspace of tt_topk_rows_ws_size bytes (0 when the rows
 * are short) long rows run in two stages (chunks in parallel, then a merge), so a row is not left
 * to one workgroup; ws = NULL takes tt_topk_rows's one-workgroup-per-row form. */
size_t tt_topk_rows_ws_size(int64_t nrows, int64_t ncols, int k);
int tt_topk_rows_ex(const float* scores, int64_t nrows, int64_t ncols, int k, void* ws, size_t ws_bytes,
                    float* out_vals, int64_t* out_idx, tt_stream_t stream);

/* ---- device-resident batch feeder (TripletDataset.__getitem__ + DataLoader collate,
 * twotower/dataset.py:262-285, twotower/train.py:411-417): dst[r, :L] = src[idx[r], :L] for int32
 * id rows; an index outside [0, n_src) yields an all-padding row and sets *bad to 1 (caller zeroes). */
int tt_gather_rows_i32(const int32_t* src, int64_t ld_src, int64_t n_src, const int64_t* idx, int64_t n, int L,
                       int32_t* dst, int64_t ld_dst, int* bad, tt_stream_t stream);
/* tt_gather_rows_i32_ex: nfield such gathers in one launch (field f reads src + f * src_field and
 * writes dst + f * dst_field: the (q, d+, d-) rows of a batch); a bad index sets *bad to
 * max(*bad, gen), gen >= 1, so a caller passing a new gen per call tests *bad == gen instead of
 * zeroing the flag before each call. */
int tt_gather_rows_i32_ex(const int32_t* src, int64_t ld_src, int64_t n_src, int64_t src_field, int nfield,
                          const int64_t* idx, int64_t n, int L, int32_t* dst, int64_t ld_dst, int64_t dst_field,
                          int* bad, int gen, tt_stream_t stream);

/* ---- measurement (bench.py's per-op times from a replayed graph) ----
 * tt_stamp: writes the device's constant-rate wall clock (tt_wall_clock_khz ticks per ms) to
 *   *slot from a one-wave kernel on `stream`: stamps launched around an op time it in stream
 *   order, also inside a captured HIP graph (where event timing is unavailable on ROCm).
 * tt_wall_clock_khz: that clock's rate for `device` (hipDeviceAttributeWallClockRate), < 0 on error. */
int tt_stamp(uint64_t* slot, tt_stream_t stream);
int tt_wall_clock_khz(int device);
/* tt_pack_blocks: `count` (<= 8) contiguous byte blocks copied into consecutive ranges of dst
 * in one launch (TrainStep's copy of a batch into the replayed graph's packed [q; p; n] input,
 * instead of torch.cat). */
int tt_pack_blocks(const void* const* srcs, const int64_t* bytes, int count, void* dst, tt_stream_t stream);

/* ---- tower head GEMMs, H in {128, 256}, E in {64, 128, 256} (MeanPoolingTower feed_forward + F.normalize,
 * twotower/encoders.py:38-42,77): fp32 GEMMs run on the bf16 MFMA with each operand split
 * into three bf16 terms (six cross products, fp32-equivalent).
 * tt_head_split: W (N x K fp32, or its transpose) -> three bf16 planes [3][N][K]
 *   (tt_head_planes_bytes bytes);
 * tt_head_gemm: out[r, n] = epi(sum_k A[r, k] W[n, k]) for the planes of W, with
 *   epi 0: relu(. + bias)            (Linear + ReLU forward); relu_mask, if not null, receives
 *          the (out > 0) bits in an opaque tile-private layout of tt_head_relu_mask_bytes(rows)
 *   epi 1: (. + bias) / max(|row|, 1e-12), norms[r] = |row|   (Linear + F.normalize forward)
 *   epi 2: . * mask(r, n)            (ReLU backward fused into dh = dy W2; relu_mask written by
 *                                     epi 0 for the same rows)
 *   epi 3: .                         (dx = dh W1)
 *   epi 4: . + bias                  (epi 1 before its normalise pass, which the caller runs:
 *                                     tt_inbatch_l2_prep; also a plain Linear + bias, K = 64 included:
 *                                     AveragePoolingTower's projection, encoders.py:84-155)
 *   epi 5: . / bias[r]               (dx = dh W1 divided by per-row divisors, IEEE division: the
 *                                     bag backward's d_pooled / denom (encoders.py:72) formed in
 *                                     the head's epilogue; bias = denom, length rows). */
size_t tt_head_planes_bytes(int N, int K);
int tt_head_split(const float* W, int N, int K, int transpose, void* planes, tt_stream_t stream);
/* the four plane sets of one Linear-ReLU-Linear head in one launch, each tt_head_planes_bytes(256,
 * 256) long, in the order W1, W2, W1^T, W2^T (forward operands, then backward operands) */
int tt_head_split_ff(const float* W1, const float* W2, void* planes, tt_stream_t stream);
/* the same for an E -> H head (W1 H x E, W2 H x H; E in {64, 128, 256}, H in {128, 256}): W1 (3 H E bf16), W2
 * (3 H H), W1^T (3 E H), W2^T (3 H H), consecutive.  tt_head_split_ff = tt_head_split_ff2(.., 256,
 * 256, ..). */
int tt_head_split_ff2(const float* W1, const float* W2, int E, int H, void* planes, tt_stream_t stream);
/* tt_head_wgrad: dW = G^T X (N x N, N in {128, 256}) and, if db is not null, db = column sums of
 * G, for G, X (rows x N fp32): the weight and bias gradients of a head Linear (encoders.py:38-42; autograd's
 * grad_W = grad_out^T input, grad_b = grad_out.sum(0)).  Deterministic (fixed-order slab sums). */
size_t tt_head_wgrad_ws_size(int64_t rows, int N);
int tt_head_wgrad(const float* G, const float* X, int64_t rows, int N, float* dW, float* db, void* ws,
                  size_t ws_bytes, tt_stream_t stream);
/* tt_head_wgrad_ex: the rectangular form, dW = G^T X (NG x NX) and db = colsum G for G (rows x NG),
 * X (rows x NX): NG = H in {128, 256}, NX in {64, 128, 256} -- the first Linear of a tower whose
 * embedding width E differs from H (C1's char tower: E 64, H 128; encoders.py:38-42).
 * tt_head_wgrad(.., N, ..) = tt_head_wgrad_ex(.., N, N, ..). */
size_t tt_head_wgrad_ex_ws_size(int64_t rows, int NG, int NX);
int tt_head_wgrad_ex(const float* G, const float* X, int64_t rows, int NG, int NX, float* dW, float* db, void* ws,
                     size_t ws_bytes, tt_stream_t stream);
/* tt_head_wgrad2: both weight gradients of a Linear-ReLU-Linear head in one launch, as slab
 * partials in ws (tt_head_wgrad2_ws_size bytes): problem 1 (G1, X1), problem 2 (G2, X2), each
 * rows x N fp32 (N in {128, 256}); tt_head_wgrad2_reduce then writes dW1 = G1^T X1, db1 = colsum G1, dW2, db2
 * (fixed-order slab sums, deterministic).  The reduce may be queued later on another stream (the
 * partials stay in ws): train_step runs the partials on a side stream beside the table update and
 * the reduce where the optimizer joins it. */
size_t tt_head_wgrad2_ws_size(int64_t rows, int N);
int tt_head_wgrad2(const float* G1, const float* X1, const float* G2, const float* X2, int64_t rows, int N,
                   void* ws, size_t ws_bytes, tt_stream_t stream);
int tt_head_wgrad2_reduce(const void* ws, int N, float* dW1, float* db1, float* dW2, float* db2,
                          tt_stream_t stream);
/* Where gradient k (0 dW1, 1 db1, 2 dW2, 3 db2) has its slab partials in tt_head_wgrad2's ws:
 * float offset and stride between slabs; returns the slab count (< 0 on bad arguments).  With
 * these a tt_adamw_multi_ex launch forms the same sums as tt_head_wgrad2_reduce. */
int tt_head_wgrad2_parts(int N, int k, int64_t* offset, int64_t* stride);
size_t tt_head_relu_mask_bytes(int64_t rows);
size_t tt_head_gemm_ws_size(int64_t rows, int epi); /* epi 1: per-slice row sums of squares */
int tt_head_gemm(const float* A, int64_t rows, int64_t lda, int K, const void* planes, int N, int epi,
                 const float* bias, uint32_t* relu_mask, float* out, float* norms, void* ws, size_t ws_bytes,
                 tt_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* TWOTOWER_AMD_H */
