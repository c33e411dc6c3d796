/*
 * factmx — MI355X-native FACT / FACT_CLIP forward+backward, C ABI.
 *
 * The reference (lucas-t-t/FACT-CLIP) has no FFI: its hot path is a tree of
 * nn.Modules calling ATen ops.  This header is the drop-in boundary UNDER that
 * Python surface: every entry point replaces one reference op site (cited as
 * file:line relative to the reference root) and is bound from Python by
 * ctypes (fact-clip_amd/factmx/native.py; binding stub in INTEGRATION.md).
 *
 * Conventions
 *   - All tensors are caller-owned device memory (fp32), row-major
 *     "(rows, channels)" = the reference's (N, B=1, C) with the unit batch
 *     axis dropped.  Leading dimensions (ld*) are in elements.
 *   - `stream` is a hipStream_t (PyTorch's current stream).  No entry point
 *     allocates, synchronises the device or keeps global mutable state; all
 *     scratch comes from a caller workspace sized by the *_workspace_* query.
 *   - Return 0 (FX_OK) or a negative FX_ERR_*; fx_last_error() (thread-local)
 *     explains the last failure.
 */
#ifndef FACTMX_H
#define FACTMX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FX_ABI_VERSION 20

enum {
  FX_OK = 0,
  FX_ERR_SHAPE = -1,     /* bad shape / argument */
  FX_ERR_HIP = -2,       /* HIP runtime error */
  FX_ERR_UNSUPPORTED = -3
};

int fx_version(void);
const char* fx_last_error(void);
/* sizeof of the ABI structs (0 gemm_desc, 1 decoder_params, 2 mstcn_params, 3 loss_term,
 * 4 video_attn, 5 mstcn2_params) so bindings can check their layouts; -1 for an unknown id */
long long fx_struct_size(int which);

/* ------------------------------------------------------------------------
 * Generic f32 GEMM on MFMA (v_mfma_f32_32x32x2_f32, exact f32 products):
 *   C[b] = epilogue( alpha * op(A[b]) (MxK) * op(B[b]) (KxN) )
 * Operands are described by a gather descriptor so the same kernel covers
 * Linear / Conv1d(k=1) (basic.py:139,177,182; blocks.py:154,158,402,414),
 * the implicit dilated Conv1d(k=3) (basic.py:138), concatenated inputs
 * (basic.py:381-385 Y_W(cat[Y, attn_feat]); blocks.py:445 sf_merge(cat)),
 * row gathers (basic.py:642 feature_seg2frame) and all their gradients.
 *
 * An operand is a logical (R x K) matrix (R = M for A, R = N for B):
 *   trans == 0 : element (r,k) = src[r*ld + k]        (K contiguous)
 *   trans == 1 : element (r,k) = src[k*ld + r]        (R contiguous)
 * trans==0 extras: k >= k_split reads the second source ptr1 (column
 *   k-k_split, leading dim ld1); rows0/rows1 gather source rows; pos adds
 *   pos[r*ld_pos + k] for k < pos_cols (positional encoding add,
 *   basic.py:313-320).
 * conv_taps == 3 (dilated conv, zero padding per video of seq_len rows, or of the ragged
 *   row ranges seq_off when nseq > 0):
 *   trans==0: k = tap*conv_cin + c, element = src[(r + s)*ld + c]
 *   trans==1: r = tap*conv_cin + c, element = src[(k + s)*ld + c]
 *   with s = (tap-1) * conv_dil * conv_dir, zero when the shifted row leaves
 *   its video.
 * ---------------------------------------------------------------------- */
typedef struct fx_operand {
  const float* ptr;
  long long ld;
  const float* ptr1;
  long long ld1;
  int k_split;
  const int32_t* rows0;
  const int32_t* rows1;
  const float* pos;
  long long ld_pos;
  int pos_cols;
  int trans;
  int conv_taps;
  int conv_cin;
  int conv_dil;
  int conv_dir;
  int seq_len;
  long long batch_stride;
  int ones_col;               /* != 0: logical row ones_col-1 reads 1.0 (fused bias gradient) */
  const int* seq_off;         /* row-major (A) conv operand of ragged videos: host (nseq + 1) row offsets, */
  int nseq;                   /* video v owns rows [seq_off[v], seq_off[v+1]) (nseq <= 16; 0: seq_len) */
} fx_operand;

typedef struct fx_gemm_desc {
  int M, N, K, batch;
  fx_operand a, b;
  float* c;
  long long ldc;
  long long c_batch_stride;
  float alpha;
  float beta;                 /* C = ... + beta*C_old */
  const float* bias;          /* + bias[n] */
  const float* resid;         /* + resid[m*ld_resid + n] */
  long long ld_resid;
  long long resid_batch_stride;
  const float* gate;          /* * (gate[m*ld_gate+n] > 0)   (ReLU backward) */
  long long ld_gate;
  int relu;                   /* 1: ReLU on the output; 2: ReLU before the residual add */
  int c_tap_cin;              /* != 0: column n = tap*c_tap_cin + c stored at c*3 + tap */
  int split_k;                /* >1: K split over workgroups, partials in workspace */
  float* workspace;
  float* c_last_col;          /* != NULL: output column N-1 goes to c_last_col[m] (bias grad) */
  long long* dbg_stamps;      /* diagnostic builds (-DFX_STAMPS) only: per-block timestamps */
  float drop_p;               /* > 0: dropout on (alpha acc + bias [relu]) before the residual add */
  unsigned long long drop_seed; /* mask of output (b, m, n): fx_dropout index (b M + m) N + n */
  long long c_last_batch_stride; /* c_last_col of batch b at c_last_col + b*stride (0: M) */
  int b_dil_growth;           /* > 1: B's conv_dil of batch b is conv_dil * growth^b (one launch for
                                 the dilated-conv weight gradients of every layer of a stack) */
  int a_dil_b1;               /* > 0: A's conv_dil for batch 1 (two dilated convs of one input, e.g.
                                 MS-TCN++'s pair, as one batch-2 launch) */
  long long bias_batch_stride; /* bias of batch b at bias + b*stride */
} fx_gemm_desc;

int fx_gemm(const fx_gemm_desc* desc, void* stream);
long long fx_gemm_workspace_floats(const fx_gemm_desc* desc);

/* ------------------------------------------------------------------------
 * nn.Linear / Conv1d(k=1) on (M, K) rows.  Replaces basic.py:139,177,182,
 * 341-345,405-407,468-470,534-538; blocks.py:154,158,402,414.
 *   fwd: y (ldy) = act((x [+pos on the first pos_cols]) . w^T + b),
 *        w is (N, K) with row stride ldw; pos nullable (add_positional_encoding
 *        fused into the operand load, basic.py:313-320).
 *   bwd: dx (lddx) [+]= dy . w ;  dw (lddw) [+]= dy^T . x ;  db [+]= colsum(dy).
 *        Any of dx/dw/db may be NULL.  accumulate_dx / accumulate_w select
 *        += for dx and for dw/db.  db rides in the dw GEMM as a virtual
 *        all-ones column of x (no separate reduction launch).
 *        relu_out (nullable): the forward output, gates dy by (relu_out>0).
 *
 * Gradient convention of every composite backward below: weight and bias
 * gradients are ACCUMULATED (+=) into the caller's buffers (the framework
 * points them at param.grad); input gradients are written.
 * ---------------------------------------------------------------------- */
int fx_linear_fwd(const float* x, long long ldx, const float* pos, long long ldpos, int pos_cols,
                  int M, int K, const float* w, long long ldw, const float* b, float* y,
                  long long ldy, int N, int relu, void* stream);
long long fx_linear_bwd_workspace_floats(int M, int K, int N);
int fx_linear_bwd(const float* dy, long long lddy, const float* x, long long ldx, const float* w,
                  long long ldw, const float* relu_out, long long ld_relu, int M, int K, int N,
                  float* dx, long long lddx, float* dw, long long lddw, float* db, int accumulate_dx,
                  int accumulate_w, float* workspace, void* stream);

/* ------------------------------------------------------------------------
 * X2Y_map, whole layer (basic.py:349-389, kq_pos=True as built by
 * Block.create_cross_attention, blocks.py:234-240):
 *   xk = X_K(X + Xpos), xv = X_V(X), yq = Y_Q(Y + Ypos)          (Hd wide)
 *   logit (Ny, Nx) = yq . xk^T / sqrt(Hd);  attn = softmax over Nx
 *   out (Ny, outdim) = Y_W(cat[Y, attn . xv])  (concat folded into the GEMM)
 * logit and attn are outputs (the losses read them, blocks.py:363-366).
 * nvid videos stacked by rows: x_off / y_off are HOST prefix arrays (nvid+1 ints,
 * NULL when nvid == 1) of each video's X / Y rows; attention stays within a video
 * and logit / attn pack the per-video (ny_v, nx_v) blocks in video order.
 * Positional tensors cover the first *pos_cols channels (nullable).
 * bwd: dout, optional direct dlogit / dattn (Ny, Nx) -> dX, dXpos, dY, dYpos
 *   (nullable) and every weight/bias gradient (accumulated, all required).
 * drop_p > 0 (training): Y_W(dropout(cat[Y, attn . xv])) (basic.py:382), fx_dropout mask
 * index r (ydim + Hd) + c over the concatenated row, regenerated by the backward.
 * bwd: the four weight-gradient GEMMs run on the library's side stream after the attention
 * gradients exist; side_defer = 1 leaves them running there (fx_side_join), 0 joins before return.
 * has_xpos / has_ypos: bit 0 = the forward had the position input; bit 1 = ACCUMULATE (+=) the
 * position gradient into dXpos / dYpos instead of writing it (one buffer shared by every op that
 * reads the same position table, so autograd does not add the per-op gradients pairwise).
 * status (bwd, nullable): device int32 word; the one-launch f2a backward core ORs
 * FX_STATUS_X2Y_TIMEOUT into it when its grid barrier gives up (its outputs are then wrong).
 * ---------------------------------------------------------------------- */
long long fx_x2y_saved_floats(int Nx, int xdim, int Ny, int ydim, int Hd);
long long fx_x2y_workspace_floats(int Nx, int xdim, int Ny, int ydim, int Hd, int outdim, int nvid,
                                  const int* x_off, const int* y_off);
int fx_x2y_fwd(const float* X, long long ldx, int Nx, int xdim, const float* Xpos, long long ldxp,
               int xpos_cols, const float* Y, long long ldy, int Ny, int ydim, const float* Ypos,
               long long ldyp, int ypos_cols, const float* wk, const float* bk, const float* wv,
               const float* bv, const float* wq, const float* bq, const float* wy, const float* by,
               int Hd, int outdim, int nvid, const int* x_off, const int* y_off, float drop_p,
               unsigned long long seed, float* out, long long ldo, float* logit, float* attn,
               float* saved, float* workspace, void* stream);
int fx_x2y_bwd(const float* X, long long ldx, int Nx, int xdim, int xpos_cols, const float* Y,
               long long ldy, int Ny, int ydim, int ypos_cols, const float* wk, const float* wv,
               const float* wq, const float* wy, int Hd, int outdim, int nvid, const int* x_off,
               const int* y_off, float drop_p, unsigned long long seed, const float* attn,
               const float* saved, const float* dout,
               long long lddo, const float* dlogit, const float* dattn, float* dX, float* dXpos,
               float* dY, float* dYpos, float* dwk, float* dbk, float* dwv, float* dbv, float* dwq,
               float* dbq, float* dwy, float* dby, int has_xpos, int has_ypos, float* workspace,
               int side_defer, int32_t* status, void* stream);

/* ------------------------------------------------------------------------
 * Action-token decoder, whole stack in one call (post-norm, ReLU FFN):
 *   cross = 1: SCADecoder (basic.py:525-557) of SCALayer (basic.py:454-523):
 *     per layer  t1 = LN_sa(x + SA(x+qpos, x+qpos, x))
 *                t2 = LN_ca(t1 + CA(t1+qpos, mem+mpos, mem))
 *                x' = LN_ff(t2 + W2 relu(W1 t2 + b1) + b2)
 *     then the optional final LayerNorm (SCADecoder.norm) and out_linear.
 *   cross = 0: SADecoder (basic.py:561-593) of SALayer (basic.py:391-452): the same
 *     without the CA stage (SALayer.norm1 -> ln_sa, norm2 -> ln_ff).
 * Any number of tokens per video (more than 64: the self-attention runs on the attention-over-T
 * kernels in query blocks of 64); training dropout per fx_decoder_params.dropout / attn_dropout.
 * SA/CA = nn.MultiheadAttention math with nhead heads (head dim A/nhead <= 64); the
 * self-attention in-projection is the packed (3A, A) in_proj_weight, the cross one
 * separate q (A,A), k (A,Hm), v (A,Hm) weights with the packed (3A) in_proj_bias.
 * Shapes: tgt (R, A) ld, qpos (R, A) dense or NULL, mem (T, Hm) ld, mpos (T, Hm) or
 * NULL, out (R, out_dim).  nvid videos stacked by rows: video v owns token rows
 * [v*R/nvid, (v+1)*R/nvid) and memory rows [v*T/nvid, (v+1)*T/nvid) (or mem_off); attention
 * never crosses videos, every projection runs over all rows at once.
 * bwd: every weight gradient ACCUMULATES (+=) into g; dtgt, dqpos (dense (R,A)),
 * dmem, dmpos are written (each nullable; dqpos accumulated when dqpos_accumulate).
 * ---------------------------------------------------------------------- */
typedef struct fx_decoder_params {
  int A, FF, nhead, num_layers, cross, Hm, out_dim, final_norm;
  float eps;
  const float* const* sa_in_w; const float* const* sa_in_b;
  const float* const* sa_out_w; const float* const* sa_out_b;
  const float* const* ca_q_w; const float* const* ca_k_w; const float* const* ca_v_w;
  const float* const* ca_in_b;
  const float* const* ca_out_w; const float* const* ca_out_b;
  const float* const* ff1_w; const float* const* ff1_b;
  const float* const* ff2_w; const float* const* ff2_b;
  const float* const* ln_sa_w; const float* const* ln_sa_b;
  const float* const* ln_ca_w; const float* const* ln_ca_b;
  const float* const* ln_ff_w; const float* const* ln_ff_b;
  const float* fn_w; const float* fn_b;
  const float* out_w; const float* out_b;
  int side_defer;             /* bwd: leave the weight-gradient GEMMs (token linears of every layer, and
                                 the frame-memory K/V projection when cross) running on the library's
                                 side stream (joined by fx_side_join), as fx_mstcn_params */
  float dropout;              /* training: nn.Dropout p of the residual branches (dropout1/2/3) and the
                                 FFN hidden layer (basic.py:444-449, 504-522); 0 = eval */
  float attn_dropout;         /* training: attention-probability dropout (MultiheadAttention dropout) */
  unsigned long long seed;    /* dropout site s of layer l: fx_dropout seed fx_drop_subseed(seed, 8 l + s),
                                 s = 0 self-attn probs, 1 its residual branch, 2 cross-attn probs,
                                 3 its residual branch, 4 FFN hidden, 5 FFN residual branch; branch masks
                                 index r * A + c (FFN hidden r * FF + c); probability masks index
                                 (query_row * nhead + head) * key_rows_total + key_row */
  const int* mem_off;         /* host (nvid + 1) frame-memory row offsets of ragged videos; NULL: video v
                                 owns memory rows [v T/nvid, (v+1) T/nvid) */
  int* status;                /* caller-owned device int32 status word (nullable): the persistent token
                                 kernel (tokdec.hip) ORs FX_STATUS_TOK_TIMEOUT into it when a grid-barrier
                                 wait gives up (outputs then wrong; never cleared by the library) */
  int dqpos_accumulate;       /* bwd: dqpos += instead of = (a position gradient shared with other ops,
                                 as fx_x2y_bwd has_xpos bit 1) */
} fx_decoder_params;

typedef struct fx_decoder_grads {
  float* const* sa_in_w; float* const* sa_in_b;
  float* const* sa_out_w; float* const* sa_out_b;
  float* const* ca_q_w; float* const* ca_k_w; float* const* ca_v_w;
  float* const* ca_in_b;
  float* const* ca_out_w; float* const* ca_out_b;
  float* const* ff1_w; float* const* ff1_b;
  float* const* ff2_w; float* const* ff2_b;
  float* const* ln_sa_w; float* const* ln_sa_b;
  float* const* ln_ca_w; float* const* ln_ca_b;
  float* const* ln_ff_w; float* const* ln_ff_b;
  float* fn_w; float* fn_b;
  float* out_w; float* out_b;
} fx_decoder_grads;

long long fx_decoder_saved_floats(const fx_decoder_params* p, int R, int T, int nvid, int has_qpos,
                                  int has_mpos);
/* One product through the persistent token kernel's GEMM phase (tokdec.hip; kernel-level tests):
 * c = epilogue(A' W^T) with A' = a (amode 0) or LayerNorm(a; ln_w, ln_b, eps 1e-5) (amode 1, K <= 256),
 * W (N, K) row-major, or with btrans W (K, N) (c = A' W); + bias, + resid (nullable).  M, N any; K a
 * multiple of 4, <= 768.  status: device int32 word (FX_STATUS_TOK_TIMEOUT). */
int fx_tok_gemm(const float* a, long long lda, int M, int N, int K, int amode, const float* ln_w, const float* ln_b,
                const float* w, long long ldw, int btrans, const float* bias, const float* resid, long long ldr,
                float* c, long long ldc, int* status, void* stream);
long long fx_decoder_workspace_floats(const fx_decoder_params* p, int R, int T, int nvid, int has_qpos,
                                      int has_mpos);
int fx_decoder_fwd(const fx_decoder_params* p, const float* tgt, long long ldt, int R, const float* qpos,
                   long long ldqp, const float* mem, long long ldm, int T, int nvid, const float* mpos,
                   long long ldmp, float* out, long long ldo, float* saved, float* workspace,
                   void* stream);
int fx_decoder_bwd(const fx_decoder_params* p, const fx_decoder_grads* g, const float* tgt,
                   long long ldt, int R, const float* qpos, const float* mem, long long ldm, int T,
                   int nvid, const float* mpos, long long ldmp, const float* dout, long long lddo, float* dtgt,
                   long long lddt, float* dqpos, float* dmem, long long lddm, float* dmpos,
                   long long lddmp, const float* saved, float* workspace, void* stream);

/* ------------------------------------------------------------------------
 * MS-TCN frame branch, whole stack in one call.
 * Replaces MSTCN.forward (basic.py:200-220) with DilatedResidualLayer.forward
 * (basic.py:154-171) unrolled over num_layers, dilation 2^i, eval-mode dropout.
 *   x (T*nvid, cin) -> y (T*nvid, cout);   hidden width F.
 *   w_in/b_in: Conv1d(cin->F, k=1) weights (nullable when in_map == 0, cin == F)
 *   w_dil[i] (F,F,3), b_dil[i], w_pw[i] (F,F,1), b_pw[i]; ln_w/ln_b[i] (nullable)
 *   w_out (cout,F,1), b_out.
 *   saved (caller-owned, fx_mstcn_saved_floats): activations kept for backward.
 * ---------------------------------------------------------------------- */
typedef struct fx_mstcn_params {
  int cin, F, cout, num_layers, layernorm, in_map;
  int dil0, dil_factor;       /* layer i dilation = dil0 * dil_factor^i (0 -> 1 and 2) */
  const float* w_in; const float* b_in;
  const float* const* w_dil; const float* const* b_dil;
  const float* const* w_pw; const float* const* b_pw;
  const float* const* ln_w; const float* const* ln_b;
  const float* w_out; const float* b_out;
  float dropout;              /* training dropout on each layer's 1x1 branch (basic.py:160); 0 = eval */
  unsigned long long seed;    /* layer i mask: fx_dropout seed fx_drop_subseed(seed, i) = seed +
                                 0xD1B54A32D192ED03 (i + 1), index row * F + channel */
  int side_defer;             /* bwd: leave the weight-gradient GEMMs running on the library's side
                                 stream (no join before return); the caller joins with fx_side_join
                                 before reading those gradients and keeps x / dy / saved / workspace
                                 alive until then (torch: record_stream on fx_side_stream()) */
  const int* seq_off;         /* ragged videos: host (nvid + 1) row offsets (video v owns rows
                                 [seq_off[v], seq_off[v+1]), zero padding at its own ends; nvid <= 16;
                                 T ignored); NULL: nvid videos of T rows */
  int fused_layers;           /* 1: the fused one-kernel layer (conv -> epilogue -> 1x1, F = 256, no LN,
                                 <= 16 ragged or uniform videos, training dropout included) where it
                                 applies and its 32-row tiles cover FX_FRL_MIN_FILL (default 80) % of
                                 the CUs (fewer rows: the two tuned GEMMs are faster); 2: wherever it
                                 applies (tests); 0: the two GEMMs per layer.  The backward's fused dX
                                 chain needs the deferred weight gradients (uniformly strided gradient
                                 buffers) when dropout is on: it keeps the masked 1x1 gradient dB_i */
} fx_mstcn_params;

typedef struct fx_mstcn_grads {
  float* w_in; float* b_in;
  float* const* w_dil; float* const* b_dil;
  float* const* w_pw; float* const* b_pw;
  float* const* ln_w; float* const* ln_b;
  float* w_out; float* b_out;
} fx_mstcn_grads;

long long fx_mstcn_saved_floats(const fx_mstcn_params* p, int rows);
/* the library's side stream of the current device (hipStream_t, created on first use; NULL on
 * failure) and the join: `stream` waits for everything enqueued on it so far */
void* fx_side_stream(void);
int fx_side_join(void* stream);
long long fx_mstcn_workspace_floats(const fx_mstcn_params* p, int rows);
int fx_mstcn_fwd(const fx_mstcn_params* p, const float* x, long long ldx, int T, int nvid,
                 float* y, long long ldy, float* saved, float* workspace, void* stream);
int fx_mstcn_bwd(const fx_mstcn_params* p, const fx_mstcn_grads* g, const float* x, long long ldx,
                 int T, int nvid, const float* dy, long long lddy, float* dx, long long lddx,
                 const float* saved, float* workspace, void* stream);

/* ------------------------------------------------------------------------
 * MSTCN2 -- the MS-TCN++ frame branch of vanilla FACT (Breakfast config, BASELINE configs[0]).
 * Replaces basic.py:222-281 MSTCN2.forward (in_map 1x1, per layer i:
 *   f' = f + dropout_i(relu(W_fu,i . cat[conv_d1,i(f), conv_d2,i(f)] + b_fu,i)),
 * conv_d1,i dilation dil_factor^(L-1-i), conv_d2,i dilation dil_factor^i, no dropout on the last
 * layer, then conv_out) for nvid stacked videos of T rows (zero padding at every video's ends).
 * Weight shapes as the reference's Conv1d (w_d*: (F, F, 3), w_fu: (F, 2F)); ngroup 1, no LN.
 * Gradients ACCUMULATE; the weight-gradient GEMMs of all layers run after the input-gradient chain
 * as batched launches on the side stream (per layer when the gradient buffers are not uniformly
 * strided).  side_defer as fx_mstcn_params.
 * ---------------------------------------------------------------------- */
typedef struct fx_mstcn2_params {
  int cin, F, cout, num_layers, in_map, dil_factor;
  const float* w_in; const float* b_in;
  const float* const* w_d1; const float* const* b_d1;
  const float* const* w_d2; const float* const* b_d2;
  const float* const* w_fu; const float* const* b_fu;
  const float* w_out; const float* b_out;
  float dropout;
  unsigned long long seed;
  int side_defer;
  const int* seq_off;         /* ragged videos, as fx_mstcn_params.seq_off */
} fx_mstcn2_params;

typedef struct fx_mstcn2_grads {
  float* w_in; float* b_in;
  float* const* w_d1; float* const* b_d1;
  float* const* w_d2; float* const* b_d2;
  float* const* w_fu; float* const* b_fu;
  float* w_out; float* b_out;
} fx_mstcn2_grads;

long long fx_mstcn2_saved_floats(const fx_mstcn2_params* p, int rows);
long long fx_mstcn2_workspace_floats(const fx_mstcn2_params* p, int rows);
int fx_mstcn2_fwd(const fx_mstcn2_params* p, const float* x, long long ldx, int T, int nvid,
                  float* y, long long ldy, float* saved, float* workspace, void* stream);
int fx_mstcn2_bwd(const fx_mstcn2_params* p, const fx_mstcn2_grads* g, const float* x, long long ldx,
                  int T, int nvid, const float* dy, long long lddy, float* dx, long long lddx,
                  const float* saved, float* workspace, void* stream);

/* ------------------------------------------------------------------------
 * Row-wise LayerNorm with fused residual (post-norm residual blocks,
 * basic.py:444-450, 504-522, 552-553; blocks.py:155; basic.py:144,166-169):
 *   y = LN(x + r) * w + b  (r nullable); optionally y = relu(y).
 *   xhat (normalised input, rows x cols) and rstd (rows) are saved for backward.
 * bwd: given dy (and the relu output if relu), returns dx (= d(x+r)),
 *   dw, db accumulated (+=) into the given buffers when non-NULL.
 * ---------------------------------------------------------------------- */
int fx_layernorm_fwd(const float* x, long long ldx, const float* r, long long ldr, const float* w,
                     const float* b, float eps, int rows, int cols, int relu, float* y, long long ldy,
                     float* xhat, long long ldxh, float* rstd, void* stream);
long long fx_layernorm_bwd_workspace_floats(int rows, int cols);
int fx_layernorm_bwd(const float* dy, long long lddy, const float* y, long long ldy, const float* xhat,
                     long long ldxh, const float* w, const float* rstd, int rows, int cols, int relu,
                     float* dx, long long lddx, float* dw, float* db, float* workspace, void* stream);

/* ------------------------------------------------------------------------
 * Row softmax family.
 * fx_softmax_rows: probs[r, :] = softmax(scale * logits[r, :]) over `cols`;
 *   used for attention (basic.py:376 X2Y softmax; MultiheadAttention).
 * fx_softmax_rows_bwd: dlogit = scale * p * (dp - sum(dp*p)) (+ dlogit_extra).
 * fx_process_feature_fwd: Block.process_feature (blocks.py:195-202):
 *   out[:, :cols-n] = x[:, :cols-n]; out[:, cols-n:] = softmax(x[:, cols-n:]);
 *   clogit (nullable, rows x n, ldc) = x[:, cols-n:] (the class logits the
 *   losses read, as a separate tensor so their gradient enters dclogit)
 * fx_process_feature_bwd: dx = [dout_feat, softmax_bwd(dout_prob) + dclogit]
 * ---------------------------------------------------------------------- */
int fx_softmax_rows(const float* logits, long long ldl, int rows, int cols, float scale,
                    float* probs, long long ldp, void* stream);
int fx_softmax_rows_bwd(const float* probs, long long ldp, const float* dprobs, long long lddp,
                        const float* dlogit_extra, long long lde, int rows, int cols, float scale,
                        float* dlogit, long long ldd, void* stream);
int fx_process_feature_fwd(const float* x, long long ldx, int rows, int cols, int n, float* out,
                           long long ldo, float* clogit, long long ldc, void* stream);
int fx_process_feature_bwd(const float* out, long long ldo, const float* dout, long long lddo,
                           const float* dclogit, long long lddc, int rows, int cols, int n, float* dx,
                           long long lddx, void* stream);

/* ------------------------------------------------------------------------
 * F.normalize(dim=-1, eps=1e-12) (blocks.py:174) and its backward.
 * ---------------------------------------------------------------------- */
int fx_l2norm_fwd(const float* x, long long ldx, int rows, int cols, float* y, long long ldy,
                  float* norm, void* stream);
int fx_l2norm_bwd(const float* y, long long ldy, const float* norm, const float* dy, long long lddy,
                  int rows, int cols, float* dx, long long lddx, void* stream);

/* ------------------------------------------------------------------------
 * Multi-head attention core (nn.MultiheadAttention math as called at
 * basic.py:442, 500, 513): per head h, P_h = softmax(Q_h K_h^T / sqrt(hd)),
 * O_h = P_h V_h.  q (Lq, E) ldq, k/v (Lk, E) ldk/ldv, o (Lq, E) ldo.
 * probs (nhead, Lq, Lk) saved for backward.  bwd gives dq, dk, dv.
 * drop_p > 0: attention dropout on P (fx_dropout mask, index (h Lq + i) Lk + j), regenerated
 * by the backward.
 * ---------------------------------------------------------------------- */
long long fx_mha_core_workspace_floats(int Lq, int Lk, int E, int nhead);
int fx_mha_core_fwd(const float* q, long long ldq, const float* k, long long ldk, const float* v,
                    long long ldv, int Lq, int Lk, int E, int nhead, float drop_p,
                    unsigned long long seed, float* probs, float* o, long long ldo, float* workspace,
                    void* stream);
int fx_mha_core_bwd(const float* q, long long ldq, const float* k, long long ldk, const float* v,
                    long long ldv, const float* probs, const float* dout, long long lddo, int Lq,
                    int Lk, int E, int nhead, float drop_p, unsigned long long seed, float* dq,
                    long long lddq, float* dk, long long lddk, float* dv, long long lddv,
                    float* workspace, void* stream);

/* ------------------------------------------------------------------------
 * Multi-head attention of a few queries over T frames, ONE fused launch for every video and
 * head (SCALayer cross-attention core, basic.py:508-516; nn.MultiheadAttention math with
 * Lq <= 64 queries and head dim hd <= 64): split-T partial softmax + P.V per workgroup, ordered
 * last-arriver merge; only lse is kept for backward (no (h, Lq, T) probabilities).
 *   nvid videos stacked by rows: queries v*Lq.., keys / values v*T..; head h = columns
 *   [h*hd, (h+1)*hd) of q, k, v, o.  fwd: o, lse (nvid, nhead, Lq).
 *   bwd: dq, dk, dv written (dk/dv may alias interleaved column ranges of one buffer).
 * ---------------------------------------------------------------------- */
long long fx_mha_t_workspace_floats(int nvid, int Lq, int T, int hd, int nhead);
int fx_mha_t_fwd(const float* q, long long ldq, const float* k, long long ldk, const float* v,
                 long long ldv, int nvid, int Lq, int T, int hd, int nhead, float scale, float* o,
                 long long ldo, float* lse, float* workspace, void* stream);
int fx_mha_t_bwd(const float* q, long long ldq, const float* k, long long ldk, const float* v,
                 long long ldv, const float* o, long long ldo, const float* dout, long long lddo,
                 const float* lse, int nvid, int Lq, int T, int hd, int nhead, float scale, float* dq,
                 long long lddq, float* dk, long long lddk, float* dv, long long lddv,
                 float* workspace, void* stream);

/* ------------------------------------------------------------------------
 * Temporal down/up-sampling (UpdateBlockTDU.temporal_downsample,
 * blocks.py:417-437; TemporalDownsampleUpsample, basic.py:595-651;
 * parse_label, utils/utils.py:25-48).
 * fx_segments_from_probs: pred[t] = argmax_c x[t, col0 + c] (first max),
 *   boundaries where pred changes, seg_id[t], seg_start[s], seg_end[s]
 *   (inclusive) and *num_seg (device int) — bit-exact run-length encoding.
 *   nvid videos of T rows each (or of the ragged host row offsets row_off, nvid + 1
 *   entries; NULL: uniform): video v's tables live at its own rows with video-local
 *   numbering, num_seg[v] its count.
 * fx_segments_globalize: after the host read num_seg: gseg_id = seg_id + the
 *   segment offset of its video; gstart/gend (sum S) = the videos' segment bounds as
 *   global frame rows, in video order.
 * fx_seg_mean_fwd: seg[s] = mean over frames of segment s (index_add / len)
 * fx_seg_mean_bwd: dframe[t] (+)= dseg[seg_id[t]] / len[seg_id[t]]
 * fx_seg_sum_rows: dseg[s] (+)= sum_{t in s} dframe[t]  (gather backward)
 * ---------------------------------------------------------------------- */
int fx_segments_from_probs(const float* x, long long ldx, int col0, int ncls, int T, int nvid,
                           const int* row_off, int32_t* pred, int32_t* seg_id, int32_t* seg_start,
                           int32_t* seg_end, int32_t* num_seg, void* stream);
int fx_segments_globalize(int nvid, int T, const int* row_off, const int32_t* num_seg_host,
                          const int32_t* seg_id, const int32_t* seg_start, const int32_t* seg_end,
                          int32_t* gseg_id, int32_t* gstart, int32_t* gend, void* stream);
int fx_seg_mean_fwd(const float* x, long long ldx, const int32_t* seg_start, const int32_t* seg_end,
                    int S, int cols, float* y, long long ldy, void* stream);
int fx_seg_mean_bwd(const float* dy, long long lddy, const int32_t* seg_id, const int32_t* seg_start,
                    const int32_t* seg_end, int T, int cols, float* dx, long long lddx, int accumulate,
                    void* stream);
int fx_seg_sum_rows(const float* dx, long long lddx, const int32_t* seg_start, const int32_t* seg_end,
                    int S, int cols, float* dy, long long lddy, int accumulate, void* stream);

/* ------------------------------------------------------------------------
 * Bidirectional single-layer GRU over the S TDU segments
 * (UpdateBlockTDU.seg_update = nn.GRU(H, H/2, 1, bidirectional=True),
 * blocks.py:401,432; PyTorch gate order r, z, n; h0 = 0).
 *   x (S, In) -> out (S, 2*Hh) = [forward h_t, backward h_t]; Hh <= 256.
 *   nseq independent sequences stacked by rows (one per video): sequence q owns rows
 *   [seq_off[q], seq_off[q+1]) (host prefix array, NULL when nseq == 1); they run concurrently.
 *   saved (fx_gru_saved_floats): per-step h_{t-1} and gates for backward.
 * relu_out != 0: out = relu([h_t fwd, h_t bwd]) (the ReLU UpdateBlockTDU applies to the GRU output,
 *   blocks.py:432, written by the recurrence kernel; the state itself stays un-rectified).
 * bwd: dout (S, 2Hh) -> dx (nullable) and every weight/bias gradient
 *   (accumulated +=; each pointer nullable); relu_y (nullable, ld ldy): the forward's rectified output,
 *   dout then flows back through the ReLU first (dout where relu_y > 0, else 0).
 * The 2 x 16 workgroups of a sequence exchange the hidden state / gate gradients
 *   through L2 with bounded spins; a peer that does not arrive within spin_max polls
 *   (0: the default, ~1 s) ends the kernel early and sets *status = FX_STATUS_GRU_TIMEOUT
 *   (status: caller-owned device int32, nullable, never cleared by the library).  The
 *   outputs are then wrong: the caller reads the word at its next host read-back and
 *   fails (factmx raises FactmxNativeError).
 * ---------------------------------------------------------------------- */
#define FX_STATUS_GRU_TIMEOUT 1
#define FX_STATUS_TOK_TIMEOUT 2   /* fx_decoder_*: a persistent token-kernel barrier wait gave up */
#define FX_STATUS_X2Y_TIMEOUT 4   /* fx_x2y_bwd: the one-launch f2a backward's grid barrier gave up */
long long fx_gru_saved_floats(int S, int Hh);
long long fx_gru_workspace_floats(int S, int nseq, int In, int Hh);
int fx_gru_bidir_fwd(const float* x, long long ldx, int S, int nseq, const int* seq_off, int In,
                     int Hh, const float* w_ih_f, const float* w_hh_f, const float* b_ih_f,
                     const float* b_hh_f, const float* w_ih_r, const float* w_hh_r, const float* b_ih_r,
                     const float* b_hh_r, float* out, long long ldo, int relu_out, float* saved,
                     float* workspace, int32_t* status, int spin_max, void* stream);
int fx_gru_bidir_bwd(const float* x, long long ldx, int S, int nseq, const int* seq_off, int In,
                     int Hh, const float* w_ih_f, const float* w_hh_f, const float* w_ih_r,
                     const float* w_hh_r, const float* saved, const float* dout, long long lddo,
                     const float* relu_y, long long ldy, float* dx, long long lddx, float* dw_ih_f, float* dw_hh_f, float* db_ih_f,
                     float* db_hh_f, float* dw_ih_r, float* dw_hh_r, float* db_ih_r, float* db_hh_r,
                     float* workspace, int32_t* status, int spin_max, void* stream);

/* ------------------------------------------------------------------------
 * Dropout (nn.Dropout in training: basic.py:158-160 MS-TCN residual branch, 382 X2Y concat,
 * MultiheadAttention probabilities, 442-450 / 504-523 decoder residual and FFN branches).
 * Counter-based mask, regenerated by every backward: element (r, c) is kept iff
 * splitmix64(seed + (r * idx_ld + idx_col0 + c + 1) * 0x9E3779B97F4A7C15) >> 32 >= p * 2^32;
 * kept values are scaled by 1 / (1 - p).  y may alias x.
 * ---------------------------------------------------------------------- */
int fx_dropout(const float* x, long long ldx, int rows, int cols, long long idx_ld, long long idx_col0,
               float p, unsigned long long seed, float* y, long long ldy, void* stream);

/* ------------------------------------------------------------------------
 * Elementwise helpers: dz = dy * (y > 0) (ReLU backward, basic.py:158,
 * blocks.py:156,414,433) and out (+)= a + b (residual merges).
 * ---------------------------------------------------------------------- */
int fx_relu_bwd(const float* dy, long long lddy, const float* y, long long ldy, int rows, int cols,
                float* dz, long long lddz, void* stream);
int fx_add(const float* a, long long lda, const float* b, long long ldb, int rows, int cols,
           float* out, long long ldo, int accumulate, void* stream);

/* ------------------------------------------------------------------------
 * Train-step tail on flat fp32 buffers (scripts/train.py:265-267:
 * torch.nn.utils.clip_grad_norm_(params, max_norm) + torch.optim.Adam.step()).
 * fx_grad_norm: workspace (fx_grad_norm_workspace_floats) <- deterministic
 *   partial sums of g^2; norm_out (nullable, 1 float) <- ||g||_2.
 * fx_clip_grad_scale: g *= min(max_norm / (||g|| + 1e-6), 1) from a workspace
 *   filled by fx_grad_norm (clip_grad_norm_ alone).
 * fx_adam_step: optional clipping (max_norm > 0: norm computed in-launch into
 *   workspace, g scaled and written back as clip_grad_norm_ leaves it), then
 *   torch.optim.Adam (amsgrad off, L2 weight_decay, bias corrections for the
 *   1-based `step`).  p, g, m, v: n floats, 16-byte aligned.
 * ---------------------------------------------------------------------- */
long long fx_grad_norm_workspace_floats(void);
int fx_grad_norm(const float* g, long long n, float* workspace, float* norm_out, void* stream);
int fx_clip_grad_scale(float* g, long long n, const float* workspace, float max_norm, void* stream);
int fx_adam_step(float* p, float* g, float* m, float* v, long long n, long long step, float lr,
                 float beta1, float beta2, float eps, float weight_decay, float max_norm,
                 float* workspace, float* norm_out, void* stream);
/* fx_adam_step_checked: the same, guarded by the device status word `status` (fx_gru_bidir_*'s
 *   status argument): when status[0] != 0 at the time the update runs -- a kernel of the step failed,
 *   e.g. a BiGRU backward timed out, so the gradients are invalid -- every block returns without
 *   touching p, g, m or v (no host synchronisation; the failure is raised on the host by the step's
 *   next status read-back).  status NULL: unguarded (= fx_adam_step). */
int fx_adam_step_checked(float* p, float* g, float* m, float* v, long long n, long long step, float lr,
                         float beta1, float beta2, float eps, float weight_decay, float max_norm,
                         float* workspace, float* norm_out, const int* status, void* stream);

/* ------------------------------------------------------------------------
 * Fused loss terms (fact_clip/models/loss.py); each returns ONE scalar
 *   out = c_ce * sum(CE terms) + c_sm * sum(smooth terms)
 * (the caller folds 1/denominator, 1/count and the term's weight into c_*; c_sm == 0 skips
 * the smooth term).  workspace: fx_loss_workspace_floats().  Backward reads the upstream
 * scalar gradient from device memory (gout) and writes the whole logit gradient.
 * fx_class_loss_*: frame_loss (loss.py:246-258) / frame_loss_tdu (260-277) with hard labels
 *   y (int64, R) or soft targets z (R, C); smooth_loss (loss.py:8-18) on the same logits
 *   (log_softmax over C, difference over rows).  x (R, C) element (r,c) at x[r*sr + c*sc];
 *   lse (R) saved by the forward; dx written dense (R, C).
 * fx_attn_loss_*: cross_attn_loss (loss.py:209-222) / cross_attn_loss_tdu (224-244): the K
 *   matched token columns a_idx (host, K <= 64) against target columns z[:, s_idx] (z dense
 *   (R, S)), per-column weights sweight (host), log_softmax over the selected columns of each
 *   row (axis 1) or over the rows of each selected column (axis 0); optional smooth_loss over
 *   all Q columns.  lse_sel ((R) for axis 1, (K) for axis 0), lse_full (R), colz (K) saved;
 *   dL written with strides (dsr, dsc).
 * ---------------------------------------------------------------------- */
long long fx_loss_workspace_floats(void);
int fx_class_loss_fwd(const float* x, long long sr, long long sc, int R, int C, const long long* y,
                      const float* z, const float* w, float c_ce, float c_sm, float* lse, float* out,
                      float* workspace, void* stream);
int fx_class_loss_bwd(const float* x, long long sr, long long sc, int R, int C, const long long* y,
                      const float* z, const float* w, const float* lse, float c_ce, float c_sm,
                      const float* gout, float* dx, void* stream);
int fx_attn_loss_fwd(const float* L, long long sr, long long sc, int R, int Q, int K,
                     const int* a_idx, const int* s_idx, const float* sweight, const float* z, int S,
                     int axis, float c_xe, float c_sm, float* lse_sel, float* lse_full, float* colz,
                     float* out, float* workspace, void* stream);
int fx_attn_loss_bwd(const float* L, long long sr, long long sc, int R, int Q, int K,
                     const int* a_idx, const int* s_idx, const float* sweight, const float* z, int S,
                     int axis, const float* lse_sel, const float* lse_full, const float* colz,
                     float c_xe, float c_sm, const float* gout, float* dL, long long dsr,
                     long long dsc, void* stream);

/* ------------------------------------------------------------------------
 * The loss phase of a batch of videos from a device-resident term table
 * (replaces MatchCriterion's per-video loss ops, loss.py:195-277, the InfoNCE
 * loss, loss.py:280-341, and their sum, blocks.py:677-786).  Each term is one
 * scalar; the caller uploads the table (terms_dev, its host copy terms_host
 * gives the shapes) and a coefficient matrix coef (nout x nterms): out[o] =
 * sum_i coef[o, i] * term_i (batch loss, per-video losses, per-block values).
 *   FX_TERM_CLASS   c_ce * sum_r sum_c z[r,c] w[c] (lse_r - x[r,c]) + c_sm * smooth
 *                   hard labels y (-1 = ignored) or, y == NULL, soft targets: row r
 *                   covers frames [rs[r], re[r]] (NULL: frame r) and z[r, gl[j]] is
 *                   its overlap with ground-truth segment j / its length
 *                   (frame_loss, frame_loss_tdu, action_token_loss, loss.py:195-277).
 *   FX_TERM_ATTN    c_ce * cross-attention CE of the K (<= FX_LOSS_MAXK) matched token columns ka
 *                   (axis 1: log_softmax over them per row, axis 0: over the rows of
 *                   each), targets = overlap(row frames, [kgs[i], kge[i]]) / row
 *                   length, column weights ksw; + c_sm * smooth over all C columns
 *                   (cross_attn_loss(_tdu), loss.py:209-244).
 *   FX_TERM_INFONCE x (R x C) <- emb . text^T * inv_temp (one GEMM), y class per
 *                   frame (-1 = held out), c_ce * (row CE mean + per-class column
 *                   log-softmax mean); backward writes demb.
 * Scratch per term: lse (R), lse2 (R + K or C), colz (K, or for InfoNCE: C counts + valid
 * frames padded to a multiple of 4, then 4 * FX_LOSS_NB * C per-row-block column partials)
 * floats; InfoNCE colz 16-byte aligned.
 * bwd: gout (nout) upstream gradient of out; every term's dx (and demb) written whole.
 * ---------------------------------------------------------------------- */
enum { FX_TERM_CLASS = 0, FX_TERM_ATTN = 1, FX_TERM_INFONCE = 2 };
#define FX_LOSS_NB 128          /* row blocks per term */
#define FX_LOSS_MAXK 512        /* matched columns of an attention term (one wave each on axis 0) */

typedef struct fx_loss_term {
  int kind, slot, R, C;
  const float* x; long long sr, sc;
  float* dx; long long dsr, dsc;
  const int32_t* y;
  const int32_t* rs; const int32_t* re;
  const int32_t* gs; const int32_t* ge; const int32_t* gl;
  int G, axis, K, D;
  const float* w;
  float c_ce, c_sm, inv_temp, pad0;
  float* lse; float* lse2; float* colz;
  const float* emb; long long ld_emb;
  const float* text;
  float* demb; long long ld_demb;
  const int32_t* ka; const int32_t* kgs; const int32_t* kge;   /* device (K): matched token columns and their */
  const float* ksw;                                            /* ground-truth segments [kgs, kge], weights */
} fx_loss_term;

long long fx_loss_terms_workspace_floats(int nterms);
int fx_loss_terms_fwd(const fx_loss_term* terms_host, const fx_loss_term* terms_dev, int nterms,
                      const float* coef, int nout, float* out, float* workspace, void* stream);
int fx_loss_terms_bwd(const fx_loss_term* terms_host, const fx_loss_term* terms_dev, int nterms,
                      const float* coef, int nout, const float* gout, float* workspace, void* stream);

/* ------------------------------------------------------------------------
 * Per-video matching cost and prediction (one launch each for every video).
 * A video: Q token class logits clogit (Q, C1) ldc; the last block's token->frame
 * attention attn (T rows, or S segment rows + seg_id (T)) lda; frame logits flogit
 * (T, C1-1) ldf (eval only); ground-truth segments gs/ge (inclusive frames) and
 * their classes gl, G of them.
 * fx_match_cost (MatchCriterion.match, loss.py:108-153 + a2f_soft_iou 91-106):
 *   cost[v, a, s] = -pc * softmax(clogit[a])[gl[s]] - a2fc * overlap / union,
 *   (nvid, Q, Gmax), s >= G_v zero-filled.
 * fx_eval_pred (Block._eval / eval_with_clip, blocks.py:243-261, 854-887):
 *   pred[pred_off + t] = argmax((1-mwt) softmax(clogit[best token of t])[:C] +
 *   mwt softmax(flogit[t])), or argmax(softmax(flogit[t])) when every token is null.
 * ---------------------------------------------------------------------- */
typedef struct fx_video_attn {
  int Q, C1, T, G;
  const float* clogit; long long ldc;
  const float* attn; long long lda;
  const int32_t* seg_id;
  const float* flogit; long long ldf;
  const int32_t* gs; const int32_t* ge; const int32_t* gl;
  long long pred_off;
} fx_video_attn;

int fx_match_cost(const fx_video_attn* vids_host, const fx_video_attn* vids_dev, int nvid, float pc,
                  float a2fc, int Gmax, float* cost, void* stream);
int fx_eval_pred(const fx_video_attn* vids_host, const fx_video_attn* vids_dev, int nvid, float mwt,
                 int32_t* pred, void* stream);

/* ------------------------------------------------------------------------
 * GEMM arithmetic precision, per caller stream (the stream every entry point
 * receives): fx_set_stream_precision(stream, prec) applies to the GEMMs later
 * enqueued on that stream; streams never set follow the library default
 * (fx_set_default_precision, initially FX_PREC_F32).  Weight-gradient GEMMs
 * (column-major A) and the small-tile / direct kernels always multiply on the
 * f32 MFMA.  FX_PREC_F32: every product on v_mfma_f32_32x32x2_f32.  FX_PREC_BF16: the
 * frame-level GEMMs with row-major operands (forward and input-gradient
 * products of the MS-TCN convs, in/out maps, projections) round their
 * operands to bf16 on the way into LDS and multiply on
 * v_mfma_f32_32x32x16_bf16, accumulating in fp32; storage, weight
 * gradients, attention, normalisation and losses stay fp32.  A performance
 * mode (BASELINE configs[1]): its deviation from the fp32 path is reported,
 * not bounded by the parity tests.  FX_PREC_F32S: the same GEMMs in fp32
 * arithmetic on the bf16 matrix cores -- each fp32 operand split into three
 * bf16 pieces (all 24 mantissa bits), the six piece products of order <= 2
 * summed in the fp32 accumulator (dropped terms < 3 * 2^-24 |a b|, the size of
 * fp32's own rounding); fp32-accurate, 2.7x the f32 MFMA rate.  FX_PREC_F32S2:
 * two pieces / three products (~2^-16 relative; measurement only).
 * ---------------------------------------------------------------------- */
enum { FX_PREC_DEFAULT = -1, FX_PREC_F32 = 0, FX_PREC_BF16 = 1, FX_PREC_F32S = 2, FX_PREC_F32S2 = 3 };
/* per stream: FX_PREC_DEFAULT clears the stream's setting (it then follows the library default) */
int fx_set_stream_precision(void* stream, int prec);
int fx_get_stream_precision(void* stream);          /* effective precision of the stream */
int fx_stream_precision_explicit(void* stream);     /* the stream's own setting, or FX_PREC_DEFAULT */
/* library default for streams without a setting (initially FX_PREC_F32) */
int fx_set_default_precision(int prec);
int fx_get_default_precision(void);

/* ----------------------------------------------------------------------
 * Profiling hooks: HIP-event timing of every launch of a kernel class
 * (bench.py roofline).  Kinds are enabled independently:
 *   0 = dilated-conv implicit GEMM (conv forward, conv dX),
 *   1 = attention over T forward (tattn_fwd_kernel + split merge),
 *   2 = attention over T backward (tattn_bwd_kernel + split merge),
 *   3-6 = X2Y cores of frame-level calls, max(Nx, Ny) >= 1024 (a2f fwd, a2f bwd, f2a fwd,
 *         f2a bwd), 11-14 = the same cores of segment-level calls,
 *   7 = fused MS-TCN layer (frl_kernel: conv + ReLU + 1x1 + residual forward,
 *       or the fused dX chain backward),
 *   8 = persistent token-kernel launches of the decoders (tokdec.hip programs),
 *   9 = SCA frame-memory K/V projection GEMM (every layer's keys and values in one
 *       frame-level product, M = frames, N = 2 d_model layers, K = memory width),
 *   10 = X2Y input projections (k, v from X, q from Y: three products per call).
 * fx_prof_enable resets one kind; fx_prof_disable resets all.
 * fx_prof_collect: the event brackets around each call (its kernels plus any host-issue gap
 *   between them).  fx_prof_collect_kernels: the same calls' kernels alone -- every kernel
 *   launched on the call's stream inside a bracket carries its own hipExtLaunchKernel event
 *   pair, i.e. its execution time as the rocprofv3 kernel trace reports it (untimed: kernels
 *   past the pool of 4 pairs per bracket; the attention and X2Y kinds only).
 * ---------------------------------------------------------------------- */
int fx_prof_enable(int kind, int max_events);
int fx_prof_collect(int kind, double* total_ms, double* total_flops, double* total_bytes,
                    int* count);
int fx_prof_collect_kernels(int kind, double* kernel_ms, int* kernels, int* untimed);
void fx_prof_disable(void);

/* Diagnostic (timeout tests): grid-barrier polls before a persistent workgroup gives up --
 * which = 0 the token kernel (fx_decoder_*), 1 the one-launch X2Y f2a backward; polls <= 0
 * restores the default (FX_TOK_SPIN or ~1 s). */
int fx_debug_set_spin(int which, int polls);

#ifdef __cplusplus
}
#endif
#endif /* FACTMX_H */
