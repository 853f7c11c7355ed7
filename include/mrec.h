/*
 * mrec.h -- C ABI of libmrec.so, the MI355X (gfx950) embedding-lookup +
 * feature-interaction hot path.
 *
 * The reference (Troublem1/PyTorchRec) is pure Python; its hot path is the ATen
 * op sites listed in SURVEY.md §2b, reached from IModel.train_step
 * (torchrec/model/IModel.py:116-125).  Each entry point below names the
 * reference interface it replaces.  The Python side (pytorchrec_amd/_mrec.py)
 * binds these with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions (all entry points):
 *   - Every buffer is a caller-owned device pointer (torch caching allocator).
 *     The library keeps no pointer past return and allocates nothing; scratch
 *     is passed in as a workspace sized by a *_workspace_size query.
 *   - Arrays documented as HOST are read during the call only.
 *   - Work is enqueued on `stream` (a hipStream_t); no call synchronises the
 *     device, so every call is safe inside hipStreamBeginCapture (hipGraphs).
 *   - Return value is an mrec_status; on error mrec_last_error() (thread-local)
 *     describes it.  No C++ exception crosses the ABI.
 *   - Out-of-range ids never fault: the kernel substitutes a zero row (forward)
 *     or skips the lookup (backward) and sets *d_oob_flag (device int32, may be
 *     NULL) to 1.  The Python wrapper turns the flag into IndexError in its
 *     checked mode, matching nn.Embedding.
 */
#ifndef MREC_H
#define MREC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MREC_ABI_VERSION 29
#define MREC_MAX_TABLES 64      /* tables per table bank / per call */
#define MREC_BWD_MAX_BATCH 8192  /* lookups per table per plan/apply call */
#define MREC_BWD_HASH_MAX_BATCH 4096  /* batches up to this use the hash plan */

typedef enum {
  MREC_OK = 0,
  MREC_EINVAL = 1, /* bad argument (null pointer, size, dtype combination) */
  MREC_EOOB = 2,   /* reserved: host-detected out-of-range id */
  MREC_EHIP = 3,   /* HIP runtime error (launch failure, ...) */
  MREC_ERCCL = 4,  /* reserved for RCCL errors */
  MREC_ENOSPC = 5  /* workspace too small */
} mrec_status;

typedef enum { MREC_F32 = 0, MREC_BF16 = 1, MREC_I32 = 2, MREC_I64 = 3 } mrec_dtype;

typedef void *mrec_stream; /* hipStream_t */

/*
 * A table bank: F embedding tables packed row-wise into one device buffer
 * [total_rows, row_stride] of `dtype`.  Table f occupies rows
 * [row_offset[f], row_offset[f] + rows[f]).  Row r holds the embedding
 * v[0..dim) and, when has_w, the first-order weight w at column `dim`
 * (SURVEY.md §7 hard part 1: "[v(16) | w | pad]").  row_stride*sizeof(dtype)
 * must be a power of two in [16, 256] bytes (64 B for bf16 D=16 + w).
 * Replaces F x torch.nn.Embedding(rows_f, dim) (+ Embedding(rows_f, 1) biases)
 * built in IModel._init_weights (FunkSVD.py:39-41, SVDPP.py:36-42).
 */
struct mrec_optim_s; /* mrec_optim: the fused row-sparse optimizer state, below */

typedef struct {
  void *data;                 /* device */
  const int64_t *row_offset;  /* HOST [n_tables] */
  const int64_t *rows;        /* HOST [n_tables] */
  int32_t n_tables;
  int32_t dim;
  int32_t row_stride; /* elements */
  int32_t has_w;
  mrec_dtype dtype; /* MREC_F32 or MREC_BF16 */
  /* HOST, may be NULL: optimizer state of the fused updates MREC_BWD_ADAGRAD /
   * _ROWWISE_ADAGRAD / _ADAM (the state belongs to the table like its rows) */
  const struct mrec_optim_s *optim;
} mrec_table_bank;

/*
 * Per-field categorical ids: field f of sample b is at
 * field_ptr[f][b * stride] (int32 or int64).  field_ptr is a HOST array of
 * n_tables device pointers, so the batch dict's per-feature tensors
 * (CategoricalColumnWithIdentity.get_feature_data, .py:20-22) are read in place
 * and a stacked [B, F] tensor is field_ptr[f] = base + f, stride = F.
 */
typedef struct {
  const void *const *field_ptr; /* HOST [n_tables] of device pointers */
  mrec_dtype dtype;             /* MREC_I32 or MREC_I64 */
  int64_t stride;               /* elements between samples */
  /* chunked addressing (0 = off): element b of a field sits at
   * field_ptr[f][(b / chunk) * chunk_stride + b % chunk] — the owner-side view of
   * an all-to-all receive buffer [source][table][slot] (see mrec_shard_*) */
  int64_t chunk;
  int64_t chunk_stride;
  int32_t pad_negative; /* negative ids are padding slots: skipped, never flagged OOB */
} mrec_ids;

int mrec_abi_version(void);
const char *mrec_last_error(void);

/* ------------------------------------------------------------------------- */
/* Forward                                                                   */
/* ------------------------------------------------------------------------- */

/*
 * Multi-table gather: out[b, f*dim + d] = bank[row_offset[f] + id[f][b], d]
 * (bit-exact copy when out_dtype == bank dtype; bf16->f32 widening is exact).
 * Row stride of `out` is out_ld elements.  If w_out != NULL (bank must have_w)
 * w_out[b*n_tables + f] = w (fp32).
 * Replaces nn.Embedding forward = aten::embedding -> index_select
 * (FunkSVD.py:47-48, NCF.py:62-65).
 */
mrec_status mrec_emb_gather_fwd(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                                void *out, mrec_dtype out_dtype, int64_t out_ld, float *w_out,
                                int32_t *d_oob_flag, mrec_stream stream);

/* flags for mrec_interact_fwd */
#define MREC_INTERACT_FM2 1         /* add 1/2 sum_d[(sum_f v)^2 - sum_f v^2] */
#define MREC_INTERACT_FIRST_ORDER 2 /* add sum_f w[id_f] (bank must have_w) */

/*
 * Fused gather + interaction + deep-input builder, one wave per sample, the
 * per-sample [F, D] block held in registers and reduced with wave shuffles:
 *   x0[b, :]   = [ v_0 .. v_{F-1} (F*dim) | dense[b, 0..n_dense) | 0 .. ]   (x0_cols wide)
 *   logit[b]   = bias + dense[b].dense_w + (FM2 ? fm2(v) : 0) + (FIRST_ORDER ? sum_f w : 0)
 *   fm_sum[b,:] = sum_f v_f   (fp32, saved for the backward; may be NULL)
 * x0 may be NULL (pure FM, config C1); dense may be NULL when n_dense==0, dense_w
 * NULL drops the dense first-order term (DCN-v2 feeds dense only to x0);
 * bias is a device float[1] (may be NULL = 0).  x0_dtype F32 or BF16.
 * Replaces: nn.Embedding gathers + torch.cat + the FM mul/sum + bias
 * embeddings (FunkSVD.py:47-51, SVDPP.py:57-66, NCF.py:62-70).
 */
mrec_status mrec_interact_fwd(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                              const float *dense, int32_t n_dense, int64_t dense_ld,
                              const float *dense_w, const float *bias, int32_t flags, void *x0,
                              mrec_dtype x0_dtype, int64_t x0_ld, int32_t x0_cols, float *logit,
                              float *fm_sum, int32_t *d_oob_flag, mrec_stream stream);

/*
 * Standalone FM second order on a dense [B, F, D] fp32 tensor (row-major),
 * y[b] = 1/2 sum_d[(sum_f v)^2 - sum_f v^2]; bwd dv = dy[b] (S_d - v_fd).
 * FunkSVD.py:51 is the F = 2 case.
 */
mrec_status mrec_fm2_fwd(const float *v, int64_t batch, int32_t fields, int32_t dim, float *y,
                         mrec_stream stream);
mrec_status mrec_fm2_bwd(const float *v, const float *dy, int64_t batch, int32_t fields,
                         int32_t dim, float *dv, mrec_stream stream);

/* ------------------------------------------------------------------------- */
/* Backward: embedding scatter-add                                           */
/* ------------------------------------------------------------------------- */

typedef enum {
  MREC_BWD_DENSE_GRAD = 0, /* grad[row] += sum g  (grad laid out like the bank, dtype of bank;
                              caller zero-fills; == aten::embedding_dense_backward) */
  MREC_BWD_SGD = 1,        /* bank[row] -= lr * sum g, round-to-nearest-even */
  MREC_BWD_SGD_SR = 2,     /* bank[row] -= lr * sum g, stochastic rounding (bf16 banks) */
  /* fused optimizers (bank->optim required; fp32 math on the row, one rounding of
   * the result into a bf16 bank).  g = the row's summed gradient this step. */
  MREC_BWD_ADAGRAD = 3,    /* torch.optim.Adagrad (lr_decay 0, initial accumulator 0, no
                              weight decay): s += g^2, w -= lr g / (sqrt(s) + eps);
                              rows not looked up are unchanged, exactly as in the dense
                              optimizer */
  MREC_BWD_ROWWISE_ADAGRAD = 4, /* one accumulator per row for the vector (s += mean_d g_d^2)
                              and one for the first-order weight: w_d -= lr g_d /
                              (sqrt(s) + eps) */
  MREC_BWD_ADAM = 5        /* dense-compatible Adam / AdamW (reference optim/AdamW.py:21-61,
                              torch.optim.Adam): a row brought from step row_step[row] to t
                              runs the zero-gradient steps it missed (momentum decay, L2
                              decay, decoupled decay) in order, then step t with g; rows
                              not looked up catch up at their next lookup or at
                              mrec_emb_optim_flush, after which the table and state equal
                              dense Adam's */
} mrec_bwd_mode;

#define MREC_OPT_DECOUPLED_WD 1       /* AdamW: w -= lr * wd * w after the step (reference
                                         AdamW.py:58-59), eps added to sqrt(v) before the
                                         bias correction of the step size (AdamW.py:50-56);
                                         else torch.optim.Adam: L2 decay g += wd * w, eps
                                         after sqrt(v / (1 - beta2^t)) */
#define MREC_OPT_NO_BIAS_CORRECTION 2 /* AdamW(correct_bias=False) */

typedef struct mrec_optim_s {
  int32_t kind;        /* the optimizer's mrec_bwd_mode (ADAGRAD / ROWWISE_ADAGRAD / ADAM) */
  float lr;            /* ADAM: lr of the zero-gradient catch-up steps run when a stale row is
                          READ (forward gathers); the apply's own lr argument steps the rows it
                          updates.  Exact while lr is constant: flush before changing it */
  double beta1, beta2; /* double: the bias corrections 1 - beta^t are formed in double, as the
                          dense optimizers do on the host */
  float eps, weight_decay;
  float grad_scale;   /* the optimizer sees grad_scale * g (a row-sharded owner: 1 / world) */
  int32_t flags;      /* MREC_OPT_* */
  float *state0;      /* ADAGRAD: sum of g^2 [total_rows, state_ld]; ROWWISE_ADAGRAD: [total_rows, 2]
                         (vector, first-order weight); ADAM: exp_avg [total_rows, state_ld] */
  float *state1;      /* ADAM: exp_avg_sq [total_rows, state_ld] */
  int32_t *row_step;  /* ADAM: the step each row is current to [total_rows] (zero at start) */
  const int64_t *d_t; /* ADAM: device step counter t, advanced by the caller before each step's
                         apply (stream-ordered, so it stays correct under graph replay) */
  int64_t state_ld;   /* floats per state row: mrec_emb_optim_state_ld */
} mrec_optim;

/* floats per optimizer-state row for a bank of `dim` (+ first-order weight) */
int64_t mrec_emb_optim_state_ld(int32_t dim, int32_t has_w);

/*
 * MREC_BWD_ADAM: bring every row not updated at the current step t (*d_t) up to t
 * by zero-gradient steps, so the table and state equal dense Adam's (call before
 * evaluation, checkpointing or a change of lr).  Other modes: no-op.
 */
mrec_status mrec_emb_optim_flush(const mrec_table_bank *bank, mrec_bwd_mode mode, float lr,
                                 mrec_stream stream);

/*
 * Bytes of workspace mrec_emb_bwd needs for `batch` lookups per table.
 */
size_t mrec_emb_bwd_workspace_size(int32_t n_tables, int64_t batch);

/*
 * Plan of the embedding backward: per table the lookups are grouped by row (an
 * LDS hash table for batch <= MREC_BWD_HASH_MAX_BATCH, a stable LDS radix sort
 * up to MREC_BWD_MAX_BATCH).  Depends only on the ids, so it can run as soon as
 * the batch is resident (or inside another launch: mrec_interact_fwd_ex,
 * mrec_shard_gather_wire).  If d_step (device uint64, may be NULL) is given the plan
 * increments it once, so a graph replayed step after step still draws fresh
 * stochastic-rounding bits.
 *
 * Workspace layout rule (ABI 28).  The plan writes the HASH layout when batch <=
 * MREC_BWD_HASH_MAX_BATCH, or when the ids are a padded exchange view
 * (mrec_ids.pad_negative) of batch <= MREC_BWD_MAX_BATCH entries; else the SORTED
 * layout.  An apply reads the hash layout when batch <= MREC_BWD_HASH_MAX_BATCH or
 * when its gradients are given (mrec_emb_bwd_apply_given with g_occ, _wire), else
 * the sorted one.  So a padded plan of more than MREC_BWD_HASH_MAX_BATCH entries is
 * consumed only by the given-gradient applies.  Every plan entry (this one, the
 * mrec_plan_job of mrec_interact_fwd_ex / mrec_shard_gather_wire(_ex)) records
 * {layout, batch, n_tables} for its workspace address when it is issued (host side;
 * the same tag, (batch << 2) | layout, is stamped into the device headers), and every
 * apply (mrec_emb_bwd_apply, _ex, _given, _rec, _wire) returns MREC_EINVAL, with
 * mrec_last_error naming both layouts, when the workspace's last plan wrote another
 * layout, batch or table count, or when no plan was issued into it.  Batch 0 reads
 * nothing and is not checked.  (The reference's autograd backward cannot be
 * mis-paired: IModel.py:123; misuse raises: IModel.py:101-108.)
 */
mrec_status mrec_emb_bwd_plan(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                              void *workspace, size_t ws_bytes, int32_t *d_oob_flag,
                              uint64_t *d_step, mrec_stream stream);

/* an embedding-backward hash plan (arguments of mrec_emb_bwd_plan) */
typedef struct {
  const mrec_table_bank *bank;
  const mrec_ids *ids;
  int64_t batch; /* 1 .. MREC_BWD_HASH_MAX_BATCH */
  void *workspace;
  size_t ws_bytes;
  int32_t *d_oob_flag;
  uint64_t *d_step;
} mrec_plan_job;

/*
 * mrec_interact_fwd plus the embedding-backward hash plan of `plan` (may be NULL;
 * batch <= MREC_BWD_HASH_MAX_BATCH) in leading workgroups of the same launch: the
 * plan depends only on the ids, and beside the latency-bound interaction it costs
 * no kernel boundary.  Same outputs as the two calls made separately.
 */
mrec_status mrec_interact_fwd_ex(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                                 const float *dense, int32_t n_dense, int64_t dense_ld,
                                 const float *dense_w, const float *bias, int32_t flags, void *x0,
                                 mrec_dtype x0_dtype, int64_t x0_ld, int32_t x0_cols, float *logit,
                                 float *fm_sum, int32_t *d_oob_flag, const mrec_plan_job *plan,
                                 mrec_stream stream);

/*
 * The compact exchange's received rows as wire records (ABI 28): record
 * p * cap_rows + pref[p][f] + j answers slot (p * n_tables + f) * cap + j of the ids
 * message `hdr` (parts x (n_tables * cap + n_tables) int32, the per-table counts
 * last; pref[p][f] = the running sum of part p's counts of the tables before f).
 */
typedef struct {
  const void *wire;     /* [parts][cap_rows] records of rec_bytes (4-B multiple, bf16 row + w) */
  int32_t rec_bytes;
  const int32_t *hdr;   /* the ids message the sender sent (mrec_shard_bucketize_dedup) */
  int32_t parts, cap, cap_rows;
  int32_t *pref;        /* out, nullable: [parts][n_tables] prefixes (mrec_emb_bwd_apply_rec) */
  int32_t *d_overflow;  /* nullable: bit 1 set when a part's counts exceed cap_rows */
} mrec_wire_rows;

/*
 * mrec_interact_fwd_ex over the compact exchange's received records without the
 * unpack launch: `bank` is the sender's slot rows (every table = the whole
 * parts x n_tables x cap slot range, row offset 0; bf16, 64-B rows) and `ids` the
 * lookups' slots (mrec_shard_bucketize_dedup pos).  Each lookup's row is read from its
 * record and also written into its slot row -- the bytes mrec_shard_wire_unpack_ex
 * writes there (the record, zeros past it), which the sender's backward reads -- and
 * the launch writes the parts' prefixes to rows->pref.  Same outputs as
 * mrec_shard_wire_unpack_ex followed by mrec_interact_fwd_ex.  (ABI 28)
 */
mrec_status mrec_interact_fwd_rec(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                                  const float *dense, int32_t n_dense, int64_t dense_ld,
                                  const float *dense_w, const float *bias, int32_t flags, void *x0,
                                  mrec_dtype x0_dtype, int64_t x0_ld, int32_t x0_cols, float *logit,
                                  float *fm_sum, int32_t *d_oob_flag, const mrec_plan_job *plan,
                                  const mrec_wire_rows *rows, mrec_stream stream);

/*
 * Gradient sources of lookup (b, f) (each may be NULL = 0):
 *   g_v[d] = dx[b, f*dim + d]                                (dx: F32/BF16, row stride dx_ld)
 *          + dfm[b] * (fm_sum[b, d] - v[b, f*dim + d])      (FM2 backward; v read from x0)
 *   g_w    = dw[b]                                          (first-order backward)
 * Segment sums are fp32 in ascending sample order (bitwise reproducible), then
 * applied per unique row as `mode` says.  Stochastic rounding draws its bits from
 * hash(seed + *d_step, row, column) (d_step may be NULL = 0).
 * Replaces aten::embedding_dense_backward + the dense optimizer step
 * (IModel.py:120-124).
 */
mrec_status mrec_emb_bwd_apply(const mrec_table_bank *bank, int64_t batch, const void *workspace,
                               size_t ws_bytes, const void *dx, mrec_dtype dx_dtype, int64_t dx_ld,
                               const float *dfm, const float *fm_sum, const void *x0,
                               mrec_dtype x0_dtype, int64_t x0_ld, const float *dw,
                               mrec_bwd_mode mode, float lr, uint64_t seed,
                               const uint64_t *d_step, void *grad, mrec_stream stream);

/*
 * Large-batch embedding backward (more than MREC_BWD_MAX_BATCH lookups per table,
 * e.g. DIN's B x L history lookups; banks of <= 2^24 rows in total): a device-wide
 * counting sort by row (plan) and ONE update per row with the sum of all its
 * lookups (apply) — what aten::embedding_dense_backward + the optimizer step do
 * for nn.Embedding (reached from FunkSVD.py:39-41 style
 * tables), instead of one SGD step per 8192-lookup chunk.  Rows hit <= 16 times
 * are summed in ascending sample order (as mrec_emb_bwd_apply); hotter rows are
 * summed in 64-bit fixed point scaled to the row's largest gradient (exact,
 * order-independent, bitwise reproducible).  Same arguments and modes as
 * mrec_emb_bwd_plan / mrec_emb_bwd_apply; `batch` = lookups per table.
 * The first mrec_emb_bwd_large_zero_bytes() bytes of the workspace must be zero
 * before its first use (torch.zeros); every apply leaves them zero again.
 */
size_t mrec_emb_bwd_large_workspace_size(const mrec_table_bank *bank, int64_t batch);
size_t mrec_emb_bwd_large_zero_bytes(const mrec_table_bank *bank, int64_t batch);
mrec_status mrec_emb_bwd_large_plan(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                                    void *workspace, size_t ws_bytes, int32_t *d_oob_flag,
                                    mrec_stream stream);
mrec_status mrec_emb_bwd_large_apply(const mrec_table_bank *bank, int64_t batch,
                                     const void *workspace, size_t ws_bytes, const void *dx,
                                     mrec_dtype dx_dtype, int64_t dx_ld, const float *dfm,
                                     const float *fm_sum, const void *x0, mrec_dtype x0_dtype,
                                     int64_t x0_ld, const float *dw, mrec_bwd_mode mode, float lr,
                                     uint64_t seed, const uint64_t *d_step, void *grad,
                                     mrec_stream stream);
/*
 * mrec_emb_bwd_large_plan + mrec_emb_bwd_large_apply in one call (ABI 20).  For
 * batches of <= 2M lookups over banks whose rows hash into at most 512 per bucket
 * (NB = batch * n_tables / 256 buckets, a power of two <= 8192), the BUCKETED plan
 * runs: lookups are partitioned by a multiplicative hash of their row (bucket
 * histograms per 8192-lookup chunk, per-bucket prefix, scatter: no per-row global
 * atomics), then one workgroup per bucket groups its rows in LDS and updates them
 * in place — rows hit <= 16 times summed in ascending sample order by one worker,
 * 17..2048 times in 64-bit fixed point by a wave (the same arithmetic, hence the
 * same bits, as the two-call path), and longer segments through the chunked
 * fixed-point kernels.  Otherwise (or with MREC_LG_ATOMIC_PLAN set) it is the
 * two calls.  Same arguments as the two calls; same workspace.
 */
mrec_status mrec_emb_bwd_large_fused(const mrec_table_bank *bank, const mrec_ids *ids,
                                     int64_t batch, void *workspace, size_t ws_bytes,
                                     int32_t *d_oob_flag, const void *dx, mrec_dtype dx_dtype,
                                     int64_t dx_ld, const float *dfm, const float *fm_sum,
                                     const void *x0, mrec_dtype x0_dtype, int64_t x0_ld,
                                     const float *dw, mrec_bwd_mode mode, float lr, uint64_t seed,
                                     const uint64_t *d_step, void *grad, mrec_stream stream);

/*
 * Kernel clock (ABI 25, measurement only: bench.py's in-step roofline).  With a
 * buffer set, every launch of the step's hot kernels -- mrec_interact_fwd_ex (the
 * plan-fused launch), mrec_emb_bwd_apply(_ex) (hash layout), mrec_tower_fwd_bwd,
 * mrec_tower_dw -- takes the next slot (in launch order; a HIP graph captured
 * meanwhile keeps its slots) and runs a clocked instantiation of its kernel
 * (the production instantiations carry no clock code).  Every wave records its
 * start and its end (after its stores are acknowledged) into shard
 * (global wave index % MREC_KCLOCK_SHARDS) of its slot:
 * buf[slot][MREC_KCLOCK_SHARDS][MREC_KCLOCK_SHARD_U64] u64, element 0 = min start,
 * element 1 = max end, s_memrealtime (100 MHz ticks); one 128-B line per shard
 * keeps the waves' atomics apart.  The caller fills starts with ~0 and ends with
 * 0 before each run and reduces min / max over the shards.  NULL turns it off
 * (the default).  Not thread-safe; host-side counter only.
 */
#define MREC_KCLOCK_SHARDS 4096
#define MREC_KCLOCK_SHARD_U64 16
void mrec_kernel_clock(void *buf, int32_t n_slots);
int32_t mrec_kernel_clock_used(void);

/*
 * Per-lookup gradients GIVEN by the caller instead of computed from dx / dfm (the
 * owner side of the row-sharded exchange).  The lookups are an
 * exchange view (mrec_ids with chunk = the entries per part): entry b of table f
 * sits in part p = b / chunk at j = b % chunk.  Exactly one source:
 *   g_occ: fp32 rows [.., g_ld], entry (p, f, j) at row p * chunk_stride + f * chunk
 *          + j (the slot exchange's received gradient slots);
 *   wire:  records of rec_bytes (wire_dtype BF16 / F32), entry (p, f, j) at record
 *          p * cap_rows + pref[p * n_tables + f] + j (the compact exchange; an entry
 *          past its part's cap_rows records gets a zero gradient).
 */
typedef struct {
  const float *g_occ;
  int64_t g_ld;
  int64_t chunk;
  int64_t chunk_stride;
  const void *wire;
  int32_t rec_bytes;
  mrec_dtype wire_dtype;
  const int32_t *pref;
  int32_t cap_rows;
} mrec_given_grads;

/*
 * Byte offset, inside the large-batch workspace, of an int32 STICKY error word
 * (ABI 25).  The fused path's huge segments (a row hit > 2048 times) are summed in
 * one launch of three dependent phases whose work items are dequeued in phase
 * order (no co-residency assumed, so a phase wait always ends); its waits are still
 * bounded, and a wait that ran out (a hardware stall; or MREC_LG_HUGE_TEST_STALL,
 * a test-only knob that makes them unreachable) leaves the rows of that launch's
 * huge segments un-updated and sets this word to 1; a bank of more than 2^24 rows
 * (only the bucketed plan) whose bucket holds more distinct rows than its LDS hash
 * sets 2 (those rows un-updated).  No kernel clears it:
 * the caller reads it at a sync point of its choosing, raises, and zeroes it.
 */
size_t mrec_emb_bwd_large_error_offset(void);

struct mrec_gemm_call_s; /* mrec_gemm_call, defined with the GEMM entry points below */

/*
 * mrec_emb_bwd_large_fused plus up to 6 deferred split-K weight-gradient reductions
 * (phase MREC_GEMM_REDUCE, as for mrec_emb_bwd_apply_ex) run by workgroups after
 * the bucket kernel's own (ABI 24): DIN's top-tower dW reduce + fused SGD leaves
 * its standalone launch.  They must not touch what the update reads or writes.  On
 * the two-call path (and for batch 0) they run as one mrec_gemm_multi after it.
 */
mrec_status mrec_emb_bwd_large_fused_ex(const mrec_table_bank *bank, const mrec_ids *ids,
                                        int64_t batch, void *workspace, size_t ws_bytes,
                                        int32_t *d_oob_flag, const void *dx, mrec_dtype dx_dtype,
                                        int64_t dx_ld, const float *dfm, const float *fm_sum,
                                        const void *x0, mrec_dtype x0_dtype, int64_t x0_ld,
                                        const float *dw, mrec_bwd_mode mode, float lr,
                                        uint64_t seed, const uint64_t *d_step, void *grad,
                                        int32_t n_reduce, const struct mrec_gemm_call_s *reduce,
                                        mrec_stream stream);

/*
 * mrec_emb_bwd_large_fused_ex over GIVEN per-lookup gradients (ABI 25; the owner
 * side of the row-sharded exchange when an exchange view exceeds the hash plan's
 * MREC_BWD_MAX_BATCH entries per table: large W * cap, Zipf).  `ids` is the exchange
 * view of the received ids (pad_negative: padding slots skipped), `batch` its
 * entries per table.  Same sums and update arithmetic as every large-batch path.
 */
mrec_status mrec_emb_bwd_large_fused_given(const mrec_table_bank *bank, const mrec_ids *ids,
                                           int64_t batch, void *workspace, size_t ws_bytes,
                                           int32_t *d_oob_flag, const mrec_given_grads *given,
                                           mrec_bwd_mode mode, float lr, uint64_t seed,
                                           const uint64_t *d_step, void *grad, int32_t n_reduce,
                                           const struct mrec_gemm_call_s *reduce,
                                           mrec_stream stream);

/*
 * mrec_emb_bwd_apply plus up to 6 deferred split-K weight-gradient reductions
 * (mrec_gemm_call with phase MREC_GEMM_REDUCE, e.g. the first MLP layer's dW +
 * fused SGD) run by extra workgroups of the same launch.  They must not touch
 * what the apply reads or writes.  A HIP graph runs the step's kernels one after
 * another, so a reduction launched on its own costs a full kernel on the
 * critical path.
 */
mrec_status mrec_emb_bwd_apply_ex(const mrec_table_bank *bank, int64_t batch,
                                  const void *workspace, size_t ws_bytes, const void *dx,
                                  mrec_dtype dx_dtype, int64_t dx_ld, const float *dfm,
                                  const float *fm_sum, const void *x0, mrec_dtype x0_dtype,
                                  int64_t x0_ld, const float *dw, mrec_bwd_mode mode, float lr,
                                  uint64_t seed, const uint64_t *d_step, void *grad,
                                  int32_t n_reduce, const struct mrec_gemm_call_s *reduce,
                                  mrec_stream stream);

/*
 * mrec_emb_bwd_apply with the per-lookup gradient rows given directly instead of
 * derived from dx / dfm / dw (those must be NULL when g_occ is set): lookup b of
 * table f contributes g_occ[idx * g_ld + 0 .. dim(+1)), idx = b when chunk == 0,
 * else (b / chunk) * chunk_stride + f * chunk + b % chunk — the receive buffer of
 * mrec_shard_lookup_grad rows after the reverse all-to-all (fp32, g_ld % 4 == 0).
 * The owner side of a row-sharded table (SURVEY.md §8e backward).  Like
 * mrec_emb_bwd_apply_ex, up to 6 deferred weight-gradient reductions may ride along.
 */
mrec_status mrec_emb_bwd_apply_given(const mrec_table_bank *bank, int64_t batch,
                                     const void *workspace, size_t ws_bytes, const void *dx,
                                     mrec_dtype dx_dtype, int64_t dx_ld, const float *dfm,
                                     const float *fm_sum, const void *x0, mrec_dtype x0_dtype,
                                     int64_t x0_ld, const float *dw, const float *g_occ,
                                     int64_t g_ld, int64_t chunk, int64_t chunk_stride,
                                     mrec_bwd_mode mode, float lr, uint64_t seed,
                                     const uint64_t *d_step, void *grad, int32_t n_reduce,
                                     const struct mrec_gemm_call_s *reduce, mrec_stream stream);
/* The owner's apply reading the received gradient RECORDS in place (ABI 23): no
 * unpack to fp32 slots.  Entry j of part p (exchange view: b = p * chunk + j,
 * chunk = cap, chunk_stride = the int32 per part of the ids message) of table f has
 * its gradient in record p * cap_rows + pref[p * n_tables + f] + j of `wire`
 * (rec_bytes each, wire_dtype BF16 or F32, 4-B aligned; pref from
 * mrec_shard_gather_wire_ex).  Same sums, order and update as mrec_emb_bwd_apply_given
 * on the unpacked slots (bit-identical). */
mrec_status mrec_emb_bwd_apply_wire(const mrec_table_bank *bank, int64_t batch,
                                    const void *workspace, size_t ws_bytes, const void *wire,
                                    int32_t rec_bytes, mrec_dtype wire_dtype, const int32_t *pref,
                                    int32_t cap_rows, int64_t chunk, int64_t chunk_stride,
                                    mrec_bwd_mode mode, float lr, uint64_t seed,
                                    const uint64_t *d_step, void *grad, int32_t n_reduce,
                                    const struct mrec_gemm_call_s *reduce, mrec_stream stream);
/* mrec_emb_bwd_apply_wire plus the data-parallel dense SGD of an
 * mrec_sgd_table_build table (device copy; sgd_blocks workgroups) in the same
 * launch (ABI 28) */
mrec_status mrec_emb_bwd_apply_wire_sgd(const mrec_table_bank *bank, int64_t batch,
                                        const void *workspace, size_t ws_bytes, const void *wire,
                                        int32_t rec_bytes, mrec_dtype wire_dtype,
                                        const int32_t *pref, int32_t cap_rows, int64_t chunk,
                                        int64_t chunk_stride, mrec_bwd_mode mode, float lr,
                                        uint64_t seed, const uint64_t *d_step, void *grad,
                                        int32_t n_reduce, const struct mrec_gemm_call_s *reduce,
                                        const void *sgd_table, int32_t sgd_blocks,
                                        mrec_stream stream);
/* The sender's DENSE_GRAD sums written straight as wire RECORDS (ABI 26): the
 * bank is the slot rows the interaction read (ids = pos, slot s = (p * n_tables +
 * f) * cap + j); slot s's sum goes to record p * cap_rows + pref[p * n_tables + f]
 * + j of `wire` (rec_bytes each, the table dtype, 4-B aligned; pref from
 * mrec_shard_wire_unpack_ex) -- the bytes mrec_shard_wire_pack would produce from
 * a zeroed sum buffer (bit-identical), without that buffer, its zeroing or the pack
 * launch.  Entries past a part's cap_rows are dropped (the unpack flagged them).
 * Hash layout only (batch <= MREC_BWD_HASH_MAX_BATCH). */
typedef struct {
  void *wire;
  int32_t rec_bytes;
  const int32_t *pref;
  int32_t cap;
  int32_t cap_rows;
} mrec_grad_records;
mrec_status mrec_emb_bwd_apply_rec(const mrec_table_bank *bank, int64_t batch,
                                   const void *workspace, size_t ws_bytes, const void *dx,
                                   mrec_dtype dx_dtype, int64_t dx_ld, const float *dfm,
                                   const float *fm_sum, const void *x0, mrec_dtype x0_dtype,
                                   int64_t x0_ld, const float *dw, const mrec_grad_records *out,
                                   int32_t n_reduce, const struct mrec_gemm_call_s *reduce,
                                   mrec_stream stream);

/* ------------------------------------------------------------------------- */
/* Communicator (RCCL over xGMI) for the row-sharded exchange                  */
/* ------------------------------------------------------------------------- */
/*
 * SURVEY.md §8(b) B2 comm entry points: with these and the mrec_shard_* kernels a
 * binding that is not torch (cgo, JNI, a C++ trainer) runs the sharded step.  The
 * reference has no communication at all (torchrec/task/Task.py:187-190 trains on
 * one device).  RCCL is opened at run time (MREC_RCCL_LIB, else the librccl
 * already in the process, else librccl.so): MREC_ERCCL when absent.
 *
 * Rank 0 calls mrec_comm_unique_id and hands the 128 bytes to every rank by any
 * host channel; each rank (one process per GPU, its HIP device current) calls
 * mrec_comm_init.  Exchanges are equal-split all-to-alls: part p of `send` (W
 * parts of the given size) goes to rank p, part p of `recv` comes from rank p --
 * the layout of mrec_shard_bucketize / mrec_shard_gather / mrec_shard_lookup_grad
 * buffers.  Stream-ordered on the caller's stream, capturable in a HIP graph; a
 * graph that captured them must be destroyed before mrec_comm_destroy (RCCL waits
 * for it).
 */
#define MREC_COMM_ID_BYTES 128
typedef struct mrec_comm_s mrec_comm;
mrec_status mrec_comm_unique_id(void *id_out /* MREC_COMM_ID_BYTES */);
mrec_status mrec_comm_init(const void *unique_id, int32_t rank, int32_t world, mrec_comm **out);
mrec_status mrec_comm_destroy(mrec_comm *comm);
int32_t mrec_comm_world(const mrec_comm *comm);
int32_t mrec_comm_rank(const mrec_comm *comm);
/* ids of the lookups for each owner: W x per_peer int32 (mrec_shard_bucketize send_ids) */
mrec_status mrec_a2a_ids(mrec_comm *comm, const int32_t *send_ids, int32_t *recv_ids,
                         int64_t per_peer, mrec_stream stream);
/* gathered rows back to the requesters: W x bytes_per_peer (multiple of 16) */
mrec_status mrec_a2a_rows_fwd(mrec_comm *comm, const void *send_rows, void *recv_rows,
                              int64_t bytes_per_peer, mrec_stream stream);
/* per-lookup gradient rows to the owners: W x floats_per_peer fp32 */
mrec_status mrec_a2a_rows_bwd(mrec_comm *comm, const float *send_grads, float *recv_grads,
                              int64_t floats_per_peer, mrec_stream stream);
/* the data-parallel dense gradient buffer, summed over the ranks in place */
mrec_status mrec_allreduce_sum_f32(mrec_comm *comm, float *buf, int64_t n, mrec_stream stream);

/* ------------------------------------------------------------------------- */
/* Row-sharded tables (one process per GPU, W = world size)                   */
/* ------------------------------------------------------------------------- */
/*
 * Table f is split cyclically: id i lives on rank i % W as local row i / W.  Every
 * exchange buffer has W equal parts of [n_tables][cap] slots (fixed capacity per
 * (owner, table)), so the all-to-alls are equal-split, need no host sync and can be
 * captured in a HIP graph.  Padding slots hold -1.  The reference has no sharding;
 * this replaces the dense nn.Embedding of IModel._init_weights (FunkSVD.py:39-41)
 * when a table does not fit, or should not be replicated on, one GPU.
 */

/*
 * Sender side, forward.  For each table f and sample b (ascending, stable):
 * owner = id % W, slot = rank of (b) among this table's ids with that owner;
 *   send_ids[(owner * n_tables + f) * cap + slot] = id / W
 *   pos[f * batch + b] = (owner * n_tables + f) * cap + slot
 * Unused slots get -1.  An id outside [0, rows[f]) sets *d_oob_flag and gets
 * pos = -1; a slot >= cap sets *d_overflow (the caller must raise) and pos = -1.
 * One 1024-thread workgroup per table; requires (W + 1) * ceil(batch/64) <= 2048.
 */
mrec_status mrec_shard_bucketize(const mrec_ids *ids, int32_t n_tables, const int64_t *rows,
                                 int64_t batch, int32_t world, int32_t cap, int32_t *send_ids,
                                 int32_t *pos, int32_t *d_overflow, int32_t *d_oob_flag,
                                 mrec_stream stream);

/*
 * Owner side, forward: rows_out[j, :] = local bank row of recv_ids[j] (table
 * f = (j / cap) % n_tables), whole row_stride elements, zeros for padding (-1) or
 * an out-of-shard id.  recv_ids / rows_out have world * n_tables * cap entries.
 */
mrec_status mrec_shard_gather(const mrec_table_bank *local, const int32_t *recv_ids,
                              int32_t world, int32_t cap, void *rows_out, mrec_stream stream);

/*
 * Sender side, backward: the gradient row of every lookup, written where its
 * embedding row came from (g_out[pos[f*batch+b] * g_ld + ...], fp32):
 *   g[d] = dx[b, f*dim + d] + dfm[b] * (fm_sum[b, d] - x0[b, f*dim + d]),  g[dim] = dw[b]
 * (same terms and NULL rules as mrec_emb_bwd_apply); lookups with pos < 0 skipped.
 */
mrec_status mrec_shard_lookup_grad(int64_t batch, int32_t n_tables, int32_t dim, int32_t has_w,
                                   const int32_t *pos, const void *dx, mrec_dtype dx_dtype,
                                   int64_t dx_ld, const float *dfm, const float *fm_sum,
                                   const void *x0, mrec_dtype x0_dtype, int64_t x0_ld,
                                   const float *dw, float *g_out, int64_t g_ld,
                                   mrec_stream stream);

/*
 * Compact exchange (ABI 19).  What crosses xGMI per step is one record per
 * DISTINCT (owner, table, id) each way instead of one 64-B slot row forward and
 * one fp32 slot row back per lookup:
 *   sender  mrec_shard_bucketize_dedup -> all-to-all ids (W parts of
 *           n_tables*cap + n_tables int32: slots, then the per-table counts)
 *   owner   mrec_shard_gather_wire     -> all-to-all rows (W parts of cap_rows
 *           records of mrec_shard_wire_bytes each: bf16 dim 16 + w = 36 B)
 *   sender  mrec_shard_wire_unpack     -> rows in the slot layout of
 *           mrec_shard_gather (the interaction reads them by pos, unchanged)
 *   backward: the sender sums the gradients of the lookups of each slot (a
 *           DENSE_GRAD apply over the slot rows, fixed ascending order), packs them
 *           (mrec_shard_wire_pack, table dtype) -> all-to-all -> the owner unpacks
 *           them to fp32 slots (mrec_shard_wire_unpack, to_f32) for
 *           mrec_emb_bwd_apply_given.
 * A part's records: table f's entries at [prefix(f), prefix(f) + count(f)) with
 * prefix(f) = sum of the counts of tables < f, so cap_rows bounds the owner's
 * total over all tables (far tighter than n_tables * cap); more sets *d_overflow
 * (the caller raises; nothing is silently dropped from a valid step).
 */
mrec_status mrec_shard_bucketize_dedup(const mrec_ids *ids, int32_t n_tables, const int64_t *rows,
                                       int64_t batch, int32_t world, int32_t cap,
                                       int32_t *send_ids, int32_t *pos, int32_t *d_overflow,
                                       int32_t *d_oob_flag, mrec_stream stream);
/*
 * Batches past one workgroup's hash (ABI 25): the sender's batch is cut into
 * C = ceil(batch / chunk_batch) chunks (chunk_batch <= 8192), each its own
 * sub-sender -- part d * C + c of send_ids holds chunk c's distinct ids for owner d
 * (owner d's C parts contiguous, so the equal-split all-to-all moves W parts of
 * C * (n_tables*cap + n_tables) int32), pos addresses slot rows of W * C parts, and
 * every other compact-exchange call takes world = W * C.  An id repeated across
 * chunks takes a slot in each; the owner sums its entries in part order.
 */
mrec_status mrec_shard_bucketize_dedup_ex(const mrec_ids *ids, int32_t n_tables,
                                          const int64_t *rows, int64_t batch, int32_t world,
                                          int32_t cap, int64_t chunk_batch, int32_t *send_ids,
                                          int32_t *pos, int32_t *d_overflow, int32_t *d_oob_flag,
                                          mrec_stream stream);

/*
 * mrec_shard_bucketize_dedup_ex with `quarters` (a power of two <= 16) workgroups per
 * table and chunk (ABI 28): workgroup q takes the ids whose quarter
 * ((id * 0x9e3779b1) mod 2^32) >> (32 - log2 quarters) is q, so each inserts and
 * ranks a quarter of the distinct ids; a part's slots are quarter-major (quarter 0's
 * distinct ids in first-lookup order, then quarter 1's, ...) -- the same records and
 * sums, another slot order.  The quarters of a (table, chunk) meet once through
 * `scratch` (mrec_shard_dedup_scratch_bytes, zeroed once before first use, then kept
 * with the caller: it holds monotonic arrival tickets); a wait that times out sets bit
 * 2 of *d_overflow.  quarters = 1 is mrec_shard_bucketize_dedup_ex.
 */
size_t mrec_shard_dedup_scratch_bytes(int32_t n_tables, int64_t chunks, int32_t world,
                                      int32_t quarters);
mrec_status mrec_shard_bucketize_dedup_q(const mrec_ids *ids, int32_t n_tables,
                                         const int64_t *rows, int64_t batch, int32_t world,
                                         int32_t cap, int64_t chunk_batch, int32_t quarters,
                                         void *scratch, size_t scratch_bytes, int32_t *send_ids,
                                         int32_t *pos, int32_t *d_overflow, int32_t *d_oob_flag,
                                         mrec_stream stream);
/* bytes of one wire record: round4((dim + has_w) * element bytes) */
int32_t mrec_shard_wire_bytes(int32_t dim, int32_t has_w, mrec_dtype dtype);
/* owner: rows of the received ids (header = recv_ids) -> wire (a lazy-Adam bank's
 * rows caught up to the current step, ABI 25); 
 * plan (may be NULL, ABI 21): the owner's backward hash plan over the same received
 * ids (an exchange view, mrec_plan_job) run by leading workgroups of this launch */
mrec_status mrec_shard_gather_wire(const mrec_table_bank *local, const int32_t *recv_ids,
                                   int32_t world, int32_t cap, int32_t cap_rows, void *wire,
                                   int32_t *d_overflow, const mrec_plan_job *plan,
                                   mrec_stream stream);
/* the same, also writing pref [world][n_tables] int32: part p's table prefixes (record
 * of entry j of table f in part p = p * cap_rows + pref[p][f] + j).  The gradient
 * records the senders return have the layout of the ids they sent, so pref also
 * addresses them for mrec_emb_bwd_apply_wire (ABI 23) */
mrec_status mrec_shard_gather_wire_ex(const mrec_table_bank *local, const int32_t *recv_ids,
                                      int32_t world, int32_t cap, int32_t cap_rows, void *wire,
                                      int32_t *pref, int32_t *d_overflow,
                                      const mrec_plan_job *plan, mrec_stream stream);
/* wire records -> slot rows [(p * n_tables + f) * cap + j] (pitch slot_bytes; to_f32:
 * bf16 records widened to fp32); zero (may be NULL): zero_bytes of the same rows of a
 * second buffer are cleared (the sender's gradient sums) */
mrec_status mrec_shard_wire_unpack(const void *wire, int32_t rec_bytes, const int32_t *hdr_ids,
                                   int32_t world, int32_t n_tables, int32_t cap, int32_t cap_rows,
                                   void *slots, int64_t slot_bytes, int32_t to_f32, void *zero,
                                   int64_t zero_bytes, int32_t *d_overflow, mrec_stream stream);
/* the same, also writing pref [world][n_tables] int32 (may be NULL, ABI 26): part
 * p's table prefixes of hdr_ids' counts -- the sender's own record layout, which
 * mrec_emb_bwd_apply_rec writes the gradient records in */
mrec_status mrec_shard_wire_unpack_ex(const void *wire, int32_t rec_bytes, const int32_t *hdr_ids,
                                      int32_t world, int32_t n_tables, int32_t cap,
                                      int32_t cap_rows, void *slots, int64_t slot_bytes,
                                      int32_t to_f32, void *zero, int64_t zero_bytes,
                                      int32_t *pref, int32_t *d_overflow, mrec_stream stream);
/* slot rows -> wire records (the first rec_bytes of each row) */
mrec_status mrec_shard_wire_pack(const void *slots, int64_t slot_bytes, int32_t rec_bytes,
                                 const int32_t *hdr_ids, int32_t world, int32_t n_tables,
                                 int32_t cap, int32_t cap_rows, void *wire, int32_t *d_overflow,
                                 mrec_stream stream);

/* ------------------------------------------------------------------------- */
/* Dense towers: MFMA bf16 GEMM with fused epilogues                          */
/* ------------------------------------------------------------------------- */

typedef enum {
  MREC_LAYOUT_ROW = 0, /* element (i, k) at ptr[i*ld + k]  (k contiguous)   */
  MREC_LAYOUT_COL = 1  /* element (i, k) at ptr[k*ld + i]  (i contiguous)   */
} mrec_layout;

typedef struct {
  const void *ptr; /* device */
  mrec_dtype dtype;
  mrec_layout layout;
  int64_t ld; /* elements */
} mrec_operand;

#define MREC_ACT_NONE 0
#define MREC_ACT_RELU 1

#define MREC_IMG_ROW_TR 0 /* bf16 weight images: row-major [N, ld] and W^T [K, ld] */
#define MREC_IMG_TOWER 1  /* MFMA-fragment images of the fused tower (mrec_tower_*) */

/* v = acc + bias[n]; aux[m,n] = v; v = act(v); v *= mul[m,n]; v += add[m,n];
 * v = (mask[m,n] > 0) ? v : 0; C = v.  Every pointer may be NULL (term skipped);
 * mul/add/aux/mask are bf16 [M, ld].  `mask` applies the ReLU' of the layer that
 * produced this GEMM's *output* operand, so a backward GEMM emits the next
 * layer's pre-activation gradient directly.  With b_ones_col the extra column (the
 * row sums of A) goes to ones_out (fp32 [M]). */
typedef struct {
  const float *bias;
  int32_t act;
  const void *mul;
  int64_t ld_mul;
  const void *add;
  int64_t ld_add;
  void *aux;
  int64_t ld_aux;
  const void *mask;
  int64_t ld_mask;
  float *ones_out;
  /* Fused SGD (update != 0; then bias/act/mul/add/aux/mask must be unset and C
   * fp32): C is a master weight updated in place, C[m, n] -= lr * v, and
   * ones_out[m] -= lr * (row sum), instead of being overwritten; the new C is
   * re-emitted as bf16 images for the next forward, img_row[m * ld_img_row + n]
   * and img_tr[n * ld_img_tr + m] (either may be NULL).  A Linear's weight-gradient
   * GEMM then IS its torch.optim.SGD step (no momentum / weight decay;
   * IModel.py:116-125) — no gradient tensor, no optimizer or conversion kernels. */
  int32_t update;
  float lr;
  void *img_row;
  int64_t ld_img_row;
  void *img_tr;
  int64_t ld_img_tr;
  /* MREC_IMG_ROW_TR: img_row / img_tr as above; MREC_IMG_TOWER: they are the
   * fwd / bwd MFMA-fragment images of mrec_tower_fwd_bwd (ld_* ignored). */
  int32_t img_kind;
} mrec_epilogue;

size_t mrec_gemm_workspace_size(int64_t M, int64_t N, int64_t K, int32_t split_k);

/*
 * C[M, N] = epi( sum_k A(m, k) B(k, n) ), A and B bf16 with 16-byte aligned rows
 * (fp32 weights go through mrec_weight_prep), fp32 accumulation on
 * v_mfma_f32_16x16x32_bf16.  Each 256-thread workgroup computes a 64x64 tile over a
 * K slice; operands are brought into LDS by global_load_lds_dwordx4 (LDS-DMA,
 * swizzled images, no register staging) through a 3-deep ring of 64-wide k
 * groups, COL operands are read back with ds_read_b64_tr_b16; K is split over
 * split_k workgroups, partials reduced in fixed order (deterministic) through
 * `workspace` (mrec_gemm_workspace_size bytes).
 * Layout ROW: element (i, k) at ptr[i*ld + k]; COL: at ptr[k*ld + i] (for B, i is
 * the output column n; nn.Linear's [out, in] weight is B in ROW layout).
 * b_ones_col == N appends a column of ones to B, so epi->ones_out[m] = sum_k A(m, k):
 * the bias gradient of a weight-gradient GEMM.  B(k, n) = 0 for b_cols <= n < N.
 * Operand pad elements between K (or the valid rows) and the next multiple of 8 must
 * be zero; C's pad columns up to min(ldc, round8(N)) are written as zero.
 * Replaces nn.Linear forward/backward = aten::addmm / mm and the ReLU
 * (Dense.py:20-24, MLP.py:22-23; SURVEY.md §2b MLP row).
 */
mrec_status mrec_gemm(int64_t M, int64_t N, int64_t K, const mrec_operand *A,
                      const mrec_operand *B, int64_t b_ones_col, int64_t b_cols,
                      const mrec_epilogue *epi, void *C, mrec_dtype c_dtype, int64_t ldc,
                      int32_t split_k, void *workspace, size_t ws_bytes, mrec_stream stream);

/* phases of a GEMM inside mrec_gemm_multi */
#define MREC_GEMM_FULL 0    /* product + epilogue (split_k must resolve to 1) */
#define MREC_GEMM_PARTIAL 1 /* split-K: fp32 partial slabs into workspace only */
#define MREC_GEMM_REDUCE 2  /* split-K: fixed-order slab reduction + epilogue only */

typedef struct mrec_gemm_call_s {
  int64_t M, N, K;
  const mrec_operand *A;
  const mrec_operand *B;
  int64_t b_ones_col;
  int64_t b_cols;
  const mrec_epilogue *epi;
  void *C;
  mrec_dtype c_dtype;
  int64_t ldc;
  int32_t split_k;
  void *workspace;
  size_t ws_bytes;
  int32_t phase; /* MREC_GEMM_* */
} mrec_gemm_call;

/*
 * Up to 4 independent GEMM phases in ONE launch (same arguments and results as
 * mrec_gemm; a split-K GEMM is run as PARTIAL in one call and REDUCE in a later one,
 * same arguments and workspace).  The calls must not depend on each other.  Used
 * for a backward layer: its dx GEMM, its dW partial slabs and the previous layer's
 * dW reduction (+ fused SGD) overlap instead of paying three launch boundaries.
 */
mrec_status mrec_gemm_multi(int32_t n, const mrec_gemm_call *calls, mrec_stream stream);



/* the CTR head's parameter finish (arguments of mrec_ctr_head_finish) */
typedef struct {
  const float *part;
  int64_t ldp;
  int64_t batch;
  int32_t H, ns;
  const float *g;
  int32_t update;
  float lr;
  float *w, *bias, *ws, *b2;
  float *dw_out, *db_out, *dws_out, *db2_out;
} mrec_head_finish_job;

/*
 * mrec_gemm_multi plus, in extra workgroups of the same launch, the CTR head
 * finish of `finish` (may be NULL).  A HIP graph runs the step's kernels one
 * after another, so a small kernel of its own sits on the critical path; beside
 * latency-bound backward GEMMs it is hidden.  Same results as
 * mrec_ctr_head_finish.  The job must be independent of the GEMM calls.
 * `plan` must be NULL (ABI 12): the embedding-backward plan rides in the
 * interaction launch (mrec_interact_fwd_ex) -- inside a GEMM launch its
 * registers held the GEMM at half occupancy -- and a plan job here is EINVAL.
 */
mrec_status mrec_gemm_multi_ex(int32_t n, const mrec_gemm_call *calls, const mrec_plan_job *plan,
                               const mrec_head_finish_job *finish, mrec_stream stream);

/*
 * fp32 [N, K] weight (row stride ldw) -> bf16 images for the GEMMs: `row`
 * [N, ldr] (B operand of the forward) and/or `tr` = W^T [K, ldt] (B operand of the
 * input-gradient GEMM); pad columns are zero.  One launch per weight per step
 * keeps the fp32 master weights as the optimizer's parameters.
 */
mrec_status mrec_weight_prep(const float *W, int64_t N, int64_t K, int64_t ldw, void *row,
                             int64_t ldr, void *tr, int64_t ldt, mrec_stream stream);

/*
 * DCN-v2 cross-network backward, elementwise stage of layer l (bf16 [M, d] rows,
 * SURVEY.md §8(a) A10): dz = g*x0; acc = (acc_init ? 0 : acc) + g*z (fp32); if
 * addend != NULL, addend = bf16(acc + g) (layer 0: its dx_l GEMM adds it and
 * yields dx0).  All rows hold round8(d) columns, 16-byte aligned; pad columns of
 * dz / acc / addend are zeroed.
 */
mrec_status mrec_dcn_cross_bwd_prep(int64_t M, int64_t d, const void *g, int64_t ldg,
                                    const void *x0, int64_t ldx0, const void *z, int64_t ldz,
                                    void *dz, int64_t lddz, float *acc, int64_t ldacc,
                                    int32_t acc_init, void *addend, int64_t ldadd,
                                    mrec_stream stream);

/*
 * Data-parallel dense update: for each job, w -= lr * g over an fp32 [N, K]
 * parameter (row strides ldw / ldg; a vector is N = 1), then the weight's bf16
 * images are re-emitted from the new w like mrec_weight_prep (`img_row` [N, ld_row]
 * and/or `img_tr` = W^T [K, ld_tr], pad columns zero; either may be NULL).  Up to
 * 16 jobs, ONE launch.  Replaces torch.optim.SGD.step() on the all-reduced
 * gradients (optimizers.py:7-11, reached from IModel.train_step, IModel.py:122-124)
 * plus a weight_prep per layer; lr already carries the 1/world of the gradient mean.
 */
typedef struct {
  float *w;
  const float *g;
  int64_t N, K, ldw, ldg;
  float lr;
  void *img_row;
  int64_t ld_row;
  void *img_tr;
  int64_t ld_tr;
  int32_t img_kind; /* MREC_IMG_ROW_TR or MREC_IMG_TOWER (see mrec_epilogue) */
} mrec_sgd_job;

mrec_status mrec_sgd_multi(int32_t n, const mrec_sgd_job *jobs, mrec_stream stream);

/*
 * The same jobs as a table another launch runs (ABI 28): mrec_sgd_table_build
 * validates them and writes the table (mrec_sgd_table_bytes() bytes, host memory)
 * and its workgroup count; the caller copies it to a 16-B aligned device buffer once
 * (it holds pointers and lr, not data) and passes that to
 * mrec_emb_bwd_apply_wire_sgd, which runs the SGD tiles beside the owner's
 * embedding update -- after the flat gradient's all-reduce, instead of a
 * mrec_sgd_multi launch of its own.  Same arithmetic, same bits.
 */
size_t mrec_sgd_table_bytes(void);
mrec_status mrec_sgd_table_build(int32_t n, const mrec_sgd_job *jobs, void *out, size_t out_bytes,
                                 int32_t *blocks);

/*
 * Fused MLP tower + CTR head + BCE loss, forward AND the input-gradient half of
 * the backward, in ONE launch (the reference's MLP =
 * Linear -> ReLU per layer (MLP.py:8-23, Dense.py:4-24), then Linear(N_L, 1) and
 * the loss of IModel.train_step (IModel.py:116-125)).  Every row of the batch is
 * independent until the weight gradients, so one 512-thread workgroup owns 16 rows
 * for the whole chain: activations stay in LDS, the bf16 weights stream from L2
 * in MFMA-fragment order (v_mfma_f32_16x16x32_bf16, fp32 accumulation), and
 *   h_l = relu(h_{l-1} W_l^T + b_l), l = 1..L (h_0 = x0);
 *   z = h_L . head_w + head_b + base + xs . ws + b2;  loss = mean BCE(z, y);
 *   dz = (sigmoid(z) - y) / batch;  dh_L = dz head_w * [h_L > 0];
 *   dh_{l-1} = (dh_l W_l) * [h_{l-1} > 0];  dx0 = dh_1 W_1.
 * Outputs (bf16 [batch, ld], pad columns zero): h_out[l] for l < L (NULL: not
 * stored), dh_out[l] for every l (the weight-gradient GEMMs' operands), dx0
 * (NULL: not stored); fp32 z, dz [batch]; the head-parameter partials (one row of
 * [dW_head (N_L) | sum dz | dws (ns)] per 16 rows, the layout
 * mrec_ctr_head_finish reduces; ceil(batch/16) rows); the loss (ticket / last
 * workgroup, deterministic, like mrec_ctr_head_fwd).
 * Weights: w_fwd[l] / w_bwd[l] are the layer's tower images (mrec_tower_weight_prep;
 * the fused SGD epilogues keep them current with img_kind = MREC_IMG_TOWER).
 * Limits: 1 <= L <= 4, every width in [1, 512], ns <= 64.
 */
typedef struct {
  int64_t batch;
  int32_t n_layers;
  int32_t width[5];          /* width[0] = x0 columns (K0), width[l] = N_l */
  const void *x0;            /* bf16 [batch, ld_x0], ld_x0 >= round8(K0), pad columns zero */
  int64_t ld_x0;
  const void *w_fwd[4];      /* bf16 tower images of W_l [N_l, N_{l-1}] */
  const void *w_bwd[4];
  const float *bias[4];      /* [N_l] (NULL: no bias) */
  const float *head_w;       /* [N_L] */
  const float *head_b;       /* [1] or NULL */
  const float *base;         /* [batch] per-sample logit added to z (FM part) or NULL */
  const float *xs;           /* side linear: xs [batch, ld_xs] fp32 . ws [ns] (+ b2) */
  int64_t ld_xs;
  int32_t ns;
  const float *ws;
  const float *b2;
  const float *y;            /* labels [batch] */
  void *h_out[4];
  int64_t ld_h[4];
  void *dh_out[4];
  int64_t ld_dh[4];
  void *dx0;
  int64_t ld_dx0;
  float *z;                  /* may be NULL */
  float *dz;
  float *part;
  int64_t ldp;               /* >= N_L + 1 + ns */
  float *loss_part;          /* [ceil(batch/16)] scratch */
  uint32_t *ticket;          /* device word, zero before the first call; left zero */
  float *loss;               /* [1] */
  /* ABI 15: kfrag != 0 -> h_out[l] / dh_out[l] are k-fragment images of [batch,
   * N_l] (mrec_kfrag_elems; ld_h / ld_dh ignored) and x0_img (may be NULL) receives
   * the k-fragment image of x0 [batch, N_0]: the operands of mrec_tower_dw */
  int32_t kfrag;
  void *x0_img;
  /* ABI 16: what runs after the forward (MREC_TOWER_*).  BCE: the loss above.
   * FORWARD: z only (h_L . head_w + head_b + base + xs . ws + b2, z required), then
   * the launch ends (no y, dz, part, loss, stores; the attention unit's scores).
   * GIVEN_DZ: dz = dz_in (no loss; y, loss_part, ticket, loss, dz may be NULL); the
   * backward as for BCE (dh_out, dx0, head partials, images). */
  int32_t mode;
  const float *dz_in;        /* [batch] for MREC_TOWER_GIVEN_DZ */
  /* ABI 27: a DCN-v2 cross network ahead of the MLP (the
   * layers are nn.Linear(d, d) as the reference's Linear init, IModel.py:61-66),
   * n_cross layers of width d = width[0], run in the same launch on the x0 block:
   *   x_0 = x0;  z_c = x_c Wc_c^T + bc_c;  x_{c+1} = x0 * z_c + x_c;  the MLP reads
   *   x_{n_cross} (its h_0);
   * backward (G_{n_cross} = the MLP's input gradient):
   *   dz_c = G_{c+1} * x0;  G_c = dz_c Wc_c + G_{c+1};
   *   dx0 = G_0 + sum_c G_{c+1} * z_c   (fp32 sum, one rounding, written to dx0).
   * With kfrag: x0_img receives x_0's image, cross_x_img[c] the image of x_{c+1}
   * (cross_x_img[n_cross - 1] is the MLP's first-layer X operand) and
   * cross_dz_img[c] that of dz_c: with them mrec_tower_dw computes dWc_c =
   * dz_c^T [x_c | 1].  z_c stays on chip (bf16) from the forward to the backward. */
  int32_t n_cross;           /* 0..3 */
  const void *cross_w_fwd[3];  /* tower images of Wc_c [d, d] */
  const void *cross_w_bwd[3];
  const float *cross_bias[3];  /* [d] (NULL: no bias) */
  void *cross_x_img[3];
  void *cross_dz_img[3];
} mrec_tower_args;

enum { MREC_TOWER_BCE = 0, MREC_TOWER_FORWARD = 1, MREC_TOWER_GIVEN_DZ = 2 };

mrec_status mrec_tower_fwd_bwd(const mrec_tower_args *a, mrec_stream stream);

/*
 * Weight gradients of the fused tower (ABI 15): for every layer l,
 *   partial slab z of dW_l [n_out, n_in + 1] = sum over K slice z of the batch of
 *   dY_l[b]^T [X_l[b] | 1]        (column n_in: the bias gradient)
 * written to ws[l] + z * n_out * ldws[l] (fp32) -- exactly the split-K PARTIAL slabs
 * of mrec_gemm(n_out, n_in, batch, dY_l COL, X_l COL, b_ones_col = n_in, ...,
 * split_k = splits), so a later mrec_gemm_multi REDUCE job of that call (same
 * workspace) finishes it (fixed-order sum + epilogue / fused SGD).  `splits` must
 * be an effective count for the batch (B = 4096: 2, 4, 5, 8, 16 ...).
 * dy_img / x_img are k-fragment images (mrec_kfrag_elems / mrec_kfrag_pack; the
 * tower writes them, mrec_tower_args.kfrag).  `finish` (may be NULL): the CTR head
 * finish in extra workgroups of the same launch (as mrec_gemm_multi_ex).
 * Replaces the weight-gradient half of autograd through nn.Linear in the
 * reference MLP (MLP.py:8-23, Dense.py:12-24) for the tower path.
 */
typedef struct {
  int32_t n_layers;          /* 1..8 (ABI 27: 8, the cross layers + the MLP) */
  int64_t batch;
  int32_t n_out[8], n_in[8];
  const void *dy_img[8];     /* bf16 k-fragment image of dY_l [batch, n_out] */
  const void *x_img[8];      /* bf16 k-fragment image of X_l [batch, n_in] */
  float *ws[8];              /* splits x n_out x ldws fp32 */
  int64_t ldws[8];           /* >= n_in + 1 (mrec_gemm's slab stride: round8(n_in + 1)) */
  int32_t splits;
} mrec_tower_dw_args;

mrec_status mrec_tower_dw(const mrec_tower_dw_args *args, const mrec_head_finish_job *finish,
                          mrec_stream stream);
/* ABI 27: + the batch feed's copy of the next record in extra workgroups (feed may be
 * NULL; see mrec_feed_job) */
struct mrec_feed_job_s; /* mrec_feed_job, defined with the batch feed below */
mrec_status mrec_tower_dw_ex(const mrec_tower_dw_args *args, const mrec_head_finish_job *finish,
                             const struct mrec_feed_job_s *feed, mrec_stream stream);

/* elements of the k-fragment image of a [rows, cols] matrix: one 1 KiB block per 16
 * columns x 32 rows, block (c / 16) * ceil(rows / 32) + r / 32, lane
 * c % 16 + 16 ((r % 32) / 8), element r % 8 (the MFMA operand order) */
int64_t mrec_kfrag_elems(int64_t rows, int64_t cols);

/* row-major bf16 [rows, cols] (row stride ld) -> its k-fragment image (pads zero) */
mrec_status mrec_kfrag_pack(const void *x, int64_t rows, int64_t cols, int64_t ld, void *img,
                            mrec_stream stream);

/* elements of the fwd (bwd = 0) or bwd (bwd = 1) tower image of an [N, K] weight */
int64_t mrec_tower_image_elems(int64_t N, int64_t K, int32_t bwd);

/* fp32 W [N, K] (row stride ldw) -> its tower images (either may be NULL).  Only
 * real elements are written: allocate the images zeroed once. */
mrec_status mrec_tower_weight_prep(const float *W, int64_t N, int64_t K, int64_t ldw,
                                   void *img_fwd, void *img_bwd, mrec_stream stream);

/* ------------------------------------------------------------------------- */
/* Batch feed                                                                 */
/* ------------------------------------------------------------------------- */

/* Copy one packed batch record (pytorchrec_amd/loader.py PackedLayout) from
 * PINNED, device-visible host memory into its device slot with a kernel on
 * `stream` (the compute queue reads the host pages over PCIe; no DMA engine, so
 * a graph launched behind it does not wait on the host).  16-B aligned, bytes a
 * multiple of 16.  Replaces the per-tensor blocking `.to(device)` of
 * IModel.train_step (torchrec/model/IModel.py:119) fed by
 * SimpleDataReader.__getitem__ (torchrec/data/SimpleDataReader.py:323-331). */
mrec_status mrec_batch_stage(void *dst, const void *host_src, int64_t bytes, mrec_stream stream);

/* ABI 27: the record at a DEVICE cursor of a pinned epoch buffer (n_records records
 * of record_bytes each, one pinned allocation): copies record d_state[0] (nothing
 * when it is past the last) into dst, then advances d_state[0] by one (d_state[1]:
 * a ticket word, zero before the first call, left zero).  Captured into a HIP graph
 * on a branch beside the train step, every replay stages the next batch while the
 * step runs (no host work per step; loader.py ColumnarLoader.capture_steps). */
mrec_status mrec_batch_stage_cursor(void *dst, const void *host_base, int64_t record_bytes,
                                    int64_t n_records, uint64_t *d_state, mrec_stream stream);

/* The same copy as a job another launch runs in extra workgroups (ABI 27:
 * mrec_tower_dw_ex), so the PCIe reads overlap that launch's work instead of taking
 * their own ~15 us on the step's critical path. */
typedef struct mrec_feed_job_s {
  void *dst;                 /* the device slot (16-B aligned) */
  const void *host_base;     /* the pinned epoch buffer: n_records x record_bytes */
  int64_t record_bytes;
  int64_t n_records;
  uint64_t *d_state;         /* [0] cursor (the record to copy, advanced by one), [1] ticket */
  /* ABI 29: the record's first widen_bytes (a multiple of 16) hold uint16 values the
   * copy writes as int32 (zero-extended): the device slot is record_bytes +
   * widen_bytes long, the rest of the record lands after the widened prefix.  The
   * loader packs ids below 65,536 this way (a third less PCIe per C2 batch); 0: a
   * plain copy */
  int64_t widen_bytes;
} mrec_feed_job;

/* ABI 29: mrec_batch_stage with a widened uint16 prefix (see mrec_feed_job) */
mrec_status mrec_batch_stage_ex(void *dst, const void *host_src, int64_t bytes, int64_t widen_bytes,
                                mrec_stream stream);
/* ABI 29: a feed job as a launch of its own (mrec_batch_stage_cursor with the job's
 * widened prefix) */
mrec_status mrec_batch_stage_job(const mrec_feed_job *job, mrec_stream stream);

/* ------------------------------------------------------------------------- */
/* CTR head and loss                                                          */
/* ------------------------------------------------------------------------- */

/*
 * z[b] = base[b] + bias[0] + h[b, :H] . w   (h bf16 rows, 16-B aligned; w fp32 [H];
 * base/bias may be NULL).  The deep tower's Linear(H, 1) (NCF.py:51, 74) fused
 * with the sum of the wide/FM logit.
 */
mrec_status mrec_head_fwd(const void *h, int64_t ldh, int64_t batch, int32_t H, const float *w,
                          const float *bias, const float *base, float *z, mrec_stream stream);
/* dh[b, :] = dz[b] * w  (bf16, pad columns up to ldh zeroed); with `mask` (bf16
 * [batch, ld_mask], may be NULL) dh[b, h] = 0 where mask[b, h] <= 0: the ReLU' of
 * the layer that produced h, so dh is that layer's pre-activation gradient. */
mrec_status mrec_head_bwd(const float *dz, const float *w, int64_t batch, int32_t H,
                          const void *mask, int64_t ld_mask, void *dh, int64_t ldh,
                          mrec_stream stream);

/*
 * torch.nn.BCEWithLogitsLoss (mean): *loss = mean(max(z,0) - z y + log1p(exp(-|z|)))
 * (fixed-order reduction); backward dz = g[0] (sigmoid(z) - y) / B (g may be NULL = 1).
 * The CTR loss the reference lacks (losses.py:8-12 has BPR/Top1/MSE only).
 */
mrec_status mrec_bce_fwd(const float *z, const float *y, int64_t batch, float *loss,
                         mrec_stream stream);
mrec_status mrec_bce_bwd(const float *z, const float *y, int64_t batch, const float *g, float *dz,
                         mrec_stream stream);

/* ------------------------------------------------------------------------- */
/* DIN target attention (config C4; absent from the reference: SURVEY.md A11) */
/* ------------------------------------------------------------------------- */
/*
 * feat[b*L + j, :] = [q_b | k_bj | q_b - k_bj | q_b * k_bj]   (bf16, 4E columns)
 * — the attention-unit input; q [B, E], k [B*L, E] bf16 (the gathered target and
 * history rows), 16-B aligned rows, E % 8 == 0, E <= 64, L <= 64.
 */
mrec_status mrec_din_feat_fwd(const void *q, int64_t ldq, const void *k, int64_t ldk,
                              int64_t batch, int32_t L, int32_t E, void *feat, int64_t ldf,
                              mrec_stream stream);
/*
 * Masked softmax pooling, one wave per sample: a_bj = softmax_j(s_bj) over valid j
 * (his[b, j] > 0 or j == 0: get_valid_his_index, torchrec/model/utils.py:5-10;
 * invalid -> -inf as scaled_dot_product_attention, SASRec.py:26-29);
 * top[b, :] = [q_b | sum_j a_bj k_bj | 0-pad] (bf16, the top MLP's input).
 * s[(b*L + j) * ld_s] fp32 scores; a [B, L] fp32 saved for the backward.
 */
mrec_status mrec_din_pool_fwd(const float *s, int64_t ld_s, const int32_t *his, int64_t ld_his,
                              const void *q, int64_t ldq, const void *k, int64_t ldk,
                              int64_t batch, int32_t L, int32_t E, float *a, void *top,
                              int64_t ldt, mrec_stream stream);
/* pooling backward from dtop[:, E:2E] = du: ds_bj = a_bj (du.k_bj - sum_i a_bi du.k_bi),
 * dk_bj = a_bj du (fp32, written) */
mrec_status mrec_din_pool_bwd(const void *dtop, int64_t lddt, const float *a, const void *k,
                              int64_t ldk, int64_t batch, int32_t L, int32_t E, float *ds,
                              float *dk, int64_t lddk, mrec_stream stream);
/* attention-unit input backward: dk_bj += df_k - df_(q-k) + df_(q*k) q_b;
 * dq_b = dtop[b, :E] + sum_j (df_q + df_(q-k) + df_(q*k) k_bj)  (position order) */
mrec_status mrec_din_feat_bwd(const void *dfeat, int64_t lddf, const void *dtop, int64_t lddt,
                              const void *q, int64_t ldq, const void *k, int64_t ldk,
                              int64_t batch, int32_t L, int32_t E, float *dk, int64_t lddk,
                              float *dq, int64_t lddq, mrec_stream stream);
/* the same, with dq and the final dk written as ONE bf16 gradient of the gathered
 * rows [target rows b < batch | history rows batch + b L + j] (row stride ld_rows;
 * dk read, not written): the gather's input gradient in the bank's dtype (ABI 15) */
mrec_status mrec_din_feat_bwd_rows(const void *dfeat, int64_t lddf, const void *dtop, int64_t lddt,
                                   const void *q, int64_t ldq, const void *k, int64_t ldk,
                                   int64_t batch, int32_t L, int32_t E, const float *dk,
                                   int64_t lddk, void *d_rows, int64_t ld_rows, mrec_stream stream);

/*
 * DIN lookup ids (ABI 17): out_item / out_cate [batch + batch L] int32 =
 * [target ids | history ids with PAD positions (his == 0 and j > 0) as -1].
 * Any other id that is negative or >= 2^31 (a target, position 0, a negative his,
 * the category of a non-PAD position) is written as INT32_MAX so that the gather's
 * range check reports it (tables must have < 2^31 - 1 rows), as nn.Embedding raises
 * IndexError on it (the reference models under torchrec/model/).
 * With mrec_ids.pad_negative set, the gather returns a zero row for -1 and the
 * embedding backward skips it: a masked history position has an exactly zero
 * gradient (softmax weight 0), so its PAD-row lookups need no update.
 * iid / cid [batch], his / hcat [batch, ld >= L], all of ids_dtype (I32 / I64).
 */
mrec_status mrec_din_lookup_ids(const void *iid, const void *cid, const void *his, int64_t ld_his,
                                const void *hcat, int64_t ld_hcat, int32_t ids_dtype,
                                int64_t batch, int32_t L, int32_t *out_item, int32_t *out_cate,
                                mrec_stream stream);

/*
 * mrec_din_lookup_ids and mrec_emb_gather_fwd (pad_negative) in ONE launch (ABI 22):
 * writes the same out_item / out_cate ids (for the embedding backward) and gathers
 * the rows of both tables into out [batch (L + 1), 2 dim] (item | category; a
 * padding slot is a zero row).  bank: the two tables (item, category), not under
 * the lazy fused Adam.  An invalid id sets *d_oob_flag (the caller raises
 * IndexError, as for nn.Embedding).  Replaces, with the ids builder, the
 * reference's nn.Embedding lookups of target and history ids (SASRec.py:85-86 idiom;
 * torchrec has no DIN).
 */
mrec_status mrec_din_gather(const mrec_table_bank *bank, const void *iid, const void *cid,
                            const void *his, int64_t ld_his, const void *hcat, int64_t ld_hcat,
                            int32_t ids_dtype, int64_t batch, int32_t L, int32_t *out_item,
                            int32_t *out_cate, void *out, mrec_dtype out_dtype, int64_t out_ld,
                            int32_t *d_oob_flag, mrec_stream stream);

/*
 * Fused DIN attention unit (ABI 17): one launch each way replaces
 * mrec_din_feat_fwd + the attention MLP's GEMMs + Linear(H2, 1) + mrec_din_pool_fwd
 * (forward) and mrec_din_pool_bwd + the GEMMs' backward + mrec_din_feat_bwd_rows
 * (backward).  Per sample, in LDS only: X = [q | k_j | q - k_j | q * k_j] (bf16),
 * s_j = w3 . relu(W2 relu(W1 x_j + b1) + b2) + b3 (bf16 MFMA operands, fp32
 * accumulation), the masked softmax / pooling of mrec_din_pool_fwd, and in the
 * backward the MLP recomputed, dX kept fp32 into the rows' gradient.
 *   rows    gathered bf16 rows [q (batch) | k (batch L)] (row stride ld_rows, 16-B
 *           aligned), his [batch, L] ids (validity: his > 0 or j == 0);
 *   w1 [H1, 4E] (ldw1), b1 [H1], w2 [H2, H1] (ldw2), b2 [H2], w3 [H2], b3 [1]:
 *           fp32 masters (nn.Linear layout; converted to bf16 in the kernel);
 *   fwd:    a [batch, L] softmax weights (saved for the backward), top [batch, ldt]
 *           = [q | u | 0-pad] bf16;
 *   bwd:    d_rows (same layout as rows) = the rows' bf16 gradient, part
 *           [parts][mrec_din_att_param_count] fp32 weight-gradient partials
 *           (parts = mrec_din_att_parts(batch));
 *   wgrad:  fixed-order sum of the partials into grads (flat [dW1 | dW2 | db1 | db2 |
 *           dw3 | db3]) or, with grads == NULL, SGD in place: p -= lr * grad.
 * Compiled shapes (mrec_din_att_supported): (E, H1, H2) with E in {16, 32} and
 * the tile counts of (32, 80, 40) (config C4) or (16, <= 32, <= 16); L <= 64.
 */
int32_t mrec_din_att_supported(int32_t E, int32_t H1, int32_t H2);
int64_t mrec_din_att_parts(int64_t batch);
int64_t mrec_din_att_param_count(int32_t E, int32_t H1, int32_t H2);
mrec_status mrec_din_att_fwd(const void *rows, int64_t ld_rows, const int32_t *his, int64_t ld_his,
                             int64_t batch, int32_t L, int32_t E, const float *w1, int64_t ldw1,
                             const float *b1, int32_t H1, const float *w2, int64_t ldw2,
                             const float *b2, int32_t H2, const float *w3, const float *b3,
                             float *a, void *top, int64_t ldt, mrec_stream stream);
mrec_status mrec_din_att_bwd(const void *rows, int64_t ld_rows, int64_t batch, int32_t L,
                             int32_t E, const float *w1, int64_t ldw1, const float *b1, int32_t H1,
                             const float *w2, int64_t ldw2, const float *b2, int32_t H2,
                             const float *w3, const float *b3, const float *a, const void *dtop,
                             int64_t lddt, void *d_rows, int64_t ld_drows, float *part,
                             int64_t parts, mrec_stream stream);
mrec_status mrec_din_att_wgrad(const float *part, int64_t parts, int32_t E, int32_t H1, int32_t H2,
                               float *grads, float lr, float *w1, int64_t ldw1, float *b1,
                               float *w2, int64_t ldw2, float *b2, float *w3, float *b3,
                               mrec_stream stream);

/*
 * Fused CTR head + BCE-with-logits (forward AND the loss gradient, one pass over h;
 * the train step of a Linear(H, 1) output layer on a ReLU MLP, the mean BCE loss):
 *   z[b]  = base[b] + bias + h[b] . w + xs[b, :ns] . ws + b2   (prediction logit;
 *           xs / ws / b2: an optional side linear term such as DeepFM's dense
 *           first-order weight and global bias, ns <= 64)
 *   dz[b] = (sigmoid(z[b]) - y[b]) / batch                       (d mean-loss / d z)
 *   dh[b, :] = dz[b] * w * (relu_mask ? h[b, :] > 0 : 1)          (bf16, pad columns 0)
 *   *loss = mean_b (max(z,0) - z y + log1p(exp(-|z|)))
 * and per-workgroup partials [dW (H) | sum dz | dws (ns)] in
 * part[mrec_ctr_head_parts(batch)][ldp >= H + 1 + ns].  The loss is reduced in the
 * same launch through loss_part[parts] and a ticket (*ticket must be 0 on entry and
 * is left 0).  H <= 1024, h / dh rows 16-byte aligned.
 * mrec_ctr_head_finish sums the partials in fixed order and, scaled by the
 * upstream gradient *g (NULL = 1), applies SGD (update: w -= lr g dW, ws -= lr g dws,
 * bias and b2 -= lr g sum dz) or writes dw_out / db_out / dws_out / db2_out.
 * Replaces Linear(H,1) + BCEWithLogitsLoss forward and backward (NCF.py:51,74 head;
 * losses.py:8-12 lacks BCE).
 */
int64_t mrec_ctr_head_parts(int64_t batch);
mrec_status mrec_ctr_head_fwd(const void *h, int64_t ldh, int64_t batch, int32_t H, const float *w,
                              const float *bias, const float *base, const float *y,
                              const float *xs, int64_t ldxs, int32_t ns, const float *ws,
                              const float *b2, int32_t relu_mask, float *z, float *dz, void *dh,
                              int64_t lddh, float *part, int64_t ldp, float *loss_part,
                              uint32_t *ticket, float *loss, mrec_stream stream);
mrec_status mrec_ctr_head_finish(const float *part, int64_t ldp, int64_t batch, int32_t H,
                                 int32_t ns, const float *g, int32_t update, float lr, float *w,
                                 float *bias, float *ws, float *b2, float *dw_out, float *db_out,
                                 float *dws_out, float *db2_out, mrec_stream stream);

/*
 * out[c] = sum_b s[b] X[b, c] for c < C, and *total = sum_b s[b] (if total != NULL):
 * the gradients of a small Linear / bias fed by per-sample scalars (dense
 * first-order weights, global bias, Linear(H, 1)).  One launch, one workgroup per
 * 8 columns, fixed-order tree reduction (deterministic).  With update != 0 the sums
 * are applied as SGD instead: out[c] -= lr * sum, *total -= lr * sum (fused
 * optimizer step of those parameters).
 */
mrec_status mrec_colsum(const float *s, const void *X, mrec_dtype x_dtype, int64_t ldx,
                        int64_t batch, int64_t C, float *out, float *total, int32_t update,
                        float lr, mrec_stream stream);

#ifdef __cplusplus
}
#endif
#endif /* MREC_H */
