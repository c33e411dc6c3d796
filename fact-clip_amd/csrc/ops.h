// Internal (non-ABI) declarations shared by the factmx translation units.
#pragma once
#include "fx_common.h"

namespace fx {

// ---- kernels (rowops.hip, segments.hip, gru.hip, gemm_f32.hip, attn_small.hip) ----
long long colsum_workspace_floats(int M, int N);
int launch_layernorm_fwd(const float* x, long long ldx, const float* r, long long ldr, const float* w,
                         const float* b, float eps, int rows, int cols, int relu, float* y, long long ldy,
                         float* mean, float* rstd, float* xhat, long long ldxh, hipStream_t s);
// the same, also writing y2 = y + pos (nullable: pos / y2 both or neither)
int launch_layernorm_fwd_pos(const float* x, long long ldx, const float* r, long long ldr, const float* w,
                             const float* b, float eps, int rows, int cols, int relu, float* y, long long ldy,
                             float* mean, float* rstd, float* xhat, long long ldxh, const float* pos, long long ldp,
                             float* y2, long long ldy2, hipStream_t s);
long long layernorm_bwd_ws_floats(int rows, int cols);
// LayerNorm weight / bias gradients of several LayerNorms in one launch: job j adds sum_rows dy * xhat to
// dw and sum_rows dy to db (either nullable), rows x cols, fixed row order (deterministic)
struct LnGradJob {
  const float* dy;
  const float* xhat;
  float* dw;
  float* db;
};
int launch_ln_param_grads(const LnGradJob* jobs, int n, int rows, int cols, long long lddy, long long ldxh,
                          hipStream_t s);
int launch_layernorm_bwd(const float* dy, long long lddy, const float* y, long long ldy, const float* xhat,
                         long long ldxh, const float* w, const float* rstd, int rows, int cols, int relu,
                         float* dx, long long lddx, float* dw, float* db, float* ws, hipStream_t s);
int launch_softmax_rows(const float* x, long long ldx, int rows, int cols, float scale, float* p, long long ldp,
                        hipStream_t s);
int launch_softmax_rows_bwd(const float* p, long long ldp, const float* dp, long long lddp, const float* extra,
                            long long lde, int rows, int cols, float scale, float* dl, long long ldd,
                            hipStream_t s);
int launch_pf_fwd(const float* x, long long ldx, int rows, int cols, int n, float* out, long long ldo, float* clogit,
                  long long ldc,
                  hipStream_t s);
int launch_pf_bwd(const float* out, long long ldo, const float* dout, long long lddo, const float* dcl,
                  long long lddc, int rows, int cols, int n, float* dx, long long lddx, hipStream_t s);
int launch_l2n_fwd(const float* x, long long ldx, int rows, int cols, float* y, long long ldy, float* nrm,
                   hipStream_t s);
int launch_l2n_bwd(const float* y, long long ldy, const float* nrm, const float* dy, long long lddy, int rows,
                   int cols, float* dx, long long lddx, hipStream_t s);
// nvid videos of T rows, or of the ragged host row offsets row_off (nvid + 1; NULL: uniform)
int launch_segments(const float* x, long long ldx, int col0, int ncls, int T, int nvid, const int* row_off,
                    int32_t* pred, int32_t* seg_id, int32_t* seg_start, int32_t* seg_end, int32_t* num_seg,
                    hipStream_t s);
int launch_seg_globalize(int nvid, int T, const int* row_off, const int32_t* num_seg_host, const int32_t* seg_id,
                         const int32_t* st, const int32_t* en, int32_t* gseg_id, int32_t* gst, int32_t* gen,
                         hipStream_t s);
int launch_seg_reduce(const float* x, long long ldx, const int32_t* st, const int32_t* en, int S, int cols, int mean,
                      float* y, long long ldy, int accumulate, hipStream_t s);
int launch_seg_mean_bwd(const float* dy, long long lddy, const int32_t* sid, const int32_t* st, const int32_t* en,
                        int T, int cols, float* dx, long long lddx, int accumulate, hipStream_t s);
// nseq independent sequences stacked by rows: sequence q owns rows [seq_off[q], seq_off[q+1]) (host)
int launch_gru_fwd(const float* gi, long long ldgi, int nseq, const int* seq_off, int Hh, const float* const whh[2],
                   const float* const bhh[2], float* out, long long ldo, int relu_out, float* saved, float* ws,
                   unsigned* status, int spin_max, hipStream_t s);
long long gru_sync_floats(int Hh, int nseq);
int launch_gru_bwd(const float* dout, long long lddo, const float* relu_y, long long ldy, int nseq, const int* seq_off,
                   int Hh, const float* const whh[2], const float* saved, float* dgi, long long lddgi, float* dgh,
                   float* sync_ws, unsigned* status, int spin_max, hipStream_t s);

// X2Y attention core with <= 64 keys per video (x2y_core.hip): logit, attn, feat in one launch;
// yoff / xoff: (nvid + 1) host row offsets, aoff: attention block offsets (ny_v * nx_v row-major each)
bool x2y_a2f_fusable(int nvid, const int* xoff, int Hd);
int launch_x2y_a2f_fwd(const float* yq, const float* xk, const float* xv, int Hd, float scale, int nvid,
                       const int* yoff, const int* xoff, const long long* aoff, float* logit, float* attn,
                       float* feat, hipStream_t s);
// long key side (f2a: <= 64 queries per video over up to T keys): chunk kernel + ordered merge; ws holds
// x2y_f2a_ws_floats(...) floats of per-chunk partials
bool x2y_f2a_fusable(int nvid, const int* xoff, const int* yoff, int Hd);
// 64-key chunks (= workgroups of the fused f2a backward passes) of a call
long long x2y_f2a_chunks(int nvid, const int* xoff);
long long x2y_f2a_ws_floats(int nvid, const int* xoff, int Hd);
int launch_x2y_f2a_fwd(const float* yq, const float* xk, const float* xv, int Hd, float scale, int nvid,
                       const int* yoff, const int* xoff, const long long* aoff, float* logit, float* attn,
                       float* feat, float* ws, hipStream_t s);
// f2a backward (dlogit, dxv, dxk, dyq of every video: the core in one launch with a grid barrier when every
// chunk's workgroup can be resident, else two, + the ordered dyq merge); ws as the forward's; status (nullable):
// FX_STATUS_X2Y_TIMEOUT when the one-launch core's barrier gives up
int launch_x2y_f2a_bwd(const float* dfeat, long long ldf, const float* xv, const float* xk, const float* yq,
                       const float* attn, const float* dattn, const float* dlogit_in, int Hd, float scale, int nvid,
                       const int* yoff, const int* xoff, const long long* aoff, float* dlogit, float* dxv, float* dxk,
                       float* dyq, float* ws, unsigned* status, hipStream_t s);
// backward, input-gradient side: dP = dfeat . xv^T (+ dattn), dlogit = attn (dP - rowsum(attn dP)) (+ dlogit_in),
// dyq = scale dlogit . xk;  dfeat rows ld ldf (16-B aligned)
// the a2f backward's weight-side products dxv = attn^T dfeat, dxk = scale dlogit^T yq in one launch
// (x2y_a2f_dw_kernel); ws: x2y_a2f_dw_ws_floats(nvid, Hd) floats
long long x2y_a2f_dw_ws_floats(int nvid, int Hd);
bool x2y_a2f_dw_ok(int nvid, const int* yoff);   // every video within the kernel's row chunks
int launch_x2y_a2f_dw(const float* attn, const float* dl, const float* dfeat, long long ldf, const float* yq, int Hd,
                      float scale, int nvid, const int* yoff, const int* xoff, const long long* aoff, float* dxv,
                      float* dxk, float* ws, hipStream_t s);
int launch_x2y_a2f_bwd(const float* dfeat, long long ldf, const float* xv, const float* xk, const float* attn,
                       const float* dattn, const float* dlogit_in, int Hd, float scale, int nvid, const int* yoff,
                       const int* xoff, const long long* aoff, float* dlogit, float* dyq, hipStream_t s);

// ---- composite helpers (capi.cpp) --------------------------------------------
int ew_grid(long long total);
int relu_bwd(const float* dy, long long lddy, const float* y, long long ldy, int rows, int cols, float* dz,
             long long lddz, hipStream_t s);
// o (+)= a + b, b added on the first bcols columns only (bcols < 0: all)
int add2(const float* a, long long lda, const float* b, long long ldb, int rows, int cols, float* o, long long ldo,
         int accumulate, hipStream_t s, int bcols = -1);
// split-K factor / workspace floats for a (M x N, depth K) product
int pick_split(int M, int N, int K, int batch = 1);
long long split_ws(int M, int N, int K, int batch = 1);
// y = (x [+pos on the first pos_cols columns]) . w^T (+b) (+relu);  w (N,K) with row stride ldw
int linear_fwd(const float* x, long long ldx, int M, int K, const float* w, const float* b, float* y, long long ldy,
               int N, int relu, hipStream_t s, long long ldw = -1, const float* pos = nullptr, long long ldpos = 0,
               int pos_cols = 0);
// dx (+)= dy . w  [* (gate > 0)];  w (N,K)
int linear_dx(const float* dy, long long lddy, const float* w, int M, int K, int N, float* dx, long long lddx,
              int accumulate, const float* gate, long long ld_gate, float* ws, hipStream_t s, long long ldw = -1);
// dw (+)= dy^T . x and db (+)= colsum(dy) in one GEMM (virtual ones column)
int linear_dwdb(const float* dy, long long lddy, const float* x, long long ldx, int M, int K, int N, float* dw,
                float* db, int accumulate, float* ws, hipStream_t s, long long lddw = -1);
int linear_dw(const float* dy, long long lddy, const float* x, long long ldx, int M, int K, int N, float* dw,
              int accumulate, float* ws, hipStream_t s, long long lddw = -1);
long long dwdb_ws(int M, int K, int N);
// the same products as descriptors, for launch_gemm_group / linear_bwd_pair
fx_gemm_desc desc_linear_dx(const float* dy, long long lddy, const float* w, int M, int K, int N, float* dx,
                            long long lddx, int accumulate, const float* gate, long long ld_gate, float* ws,
                            long long ldw = -1);
fx_gemm_desc desc_linear_dwdb(const float* dy, long long lddy, const float* x, long long ldx, int M, int K, int N,
                              float* dw, float* db, int accumulate, float* ws, long long lddw = -1);
// dW/db and dX of one linear layer from the same dY: one launch when both are direct-kernel shapes
int linear_bwd_pair(const fx_gemm_desc& dwdb, const fx_gemm_desc& dx, hipStream_t s);

// ---- fused small multi-head attention (attn_small.hip): Lq, Lk, head_dim <= 64 ----
// drop_p > 0: attention-probability dropout with attn_t.hip's mask (TAttnOpts), probs saved un-dropped
// nvid independent problems stacked by rows (video v: q/o rows v*Lq.., k/v rows v*Lk..);
// probs (nvid, nhead, Lq, Lk) saved; o (Lq, nhead*hd) with row stride ldo.
int launch_mha_small_fwd(const float* q, long long ldq, const float* k, long long ldk, const float* v,
                         long long ldv, int Lq, int Lk, int hd, int nhead, float scale, float* probs, float* o,
                         long long ldo, hipStream_t s, int nvid = 1, float drop_p = 0.f,
                         unsigned long long seed = 0);
// dq, dk, dv written (nullable) with their row strides
int launch_mha_small_bwd(const float* q, long long ldq, const float* k, long long ldk, const float* v,
                         long long ldv, const float* probs, const float* dout, long long lddo, int Lq, int Lk, int hd,
                         int nhead, float scale, float* dq, long long lddq, float* dk, long long lddk, float* dv,
                         long long lddv, hipStream_t s, int nvid = 1, float drop_p = 0.f, unsigned long long seed = 0);

// ---- fused multi-head attention of queries over T frames (attn_t.hip) ---------------------
// nvid videos stacked by rows (queries v*Qv.., keys/values v*Tv.. or opt->koff); head h = columns
// [h*hd, h*hd+hd) of q/k/v/o.  fwd writes o and lse (nvid, nhead, Qv); bwd writes (or with acc_kv adds)
// dk, dv (rows: one per key) and writes dq.  More than 64 queries run as blocks of 64.
struct TAttnOpts {
  const int* koff = nullptr;        // host (nvid + 1) key-row offsets of ragged videos; Tv = the longest
  float drop_p = 0.f;               // attention-probability dropout (training)
  unsigned long long drop_seed = 0; // mask of probability (query row qg, head h, key row kg):
                                    // fx_drop_bits(seed, (qg * nhead + h) * total_key_rows + kg)
  int acc_kv = 0;                   // bwd: dk / dv += instead of =
};
long long tattn_ws_floats(int nvid, int Qv, int Tv, int hd, int nhead);
int launch_tattn_fwd(const float* q, long long ldq, const float* k, long long ldk, const float* v, long long ldv,
                     int nvid, int Qv, int Tv, int hd, int nhead, float scale, float* o, long long ldo, float* lse,
                     float* ws, hipStream_t s, const TAttnOpts* opt = nullptr);
int launch_tattn_bwd(const float* q, long long ldq, const float* k, long long ldk, const float* v, long long ldv,
                     const float* o, long long ldo, const float* dout, long long lddo, const float* lse, int nvid,
                     int Qv, int Tv, int hd, int nhead, float scale, float* dq, long long lddq, float* dk,
                     long long lddk, float* dv, long long lddv, float* ws, hipStream_t s,
                     const TAttnOpts* opt = nullptr);

// fused MS-TCN layer step (mstcn_fused.hip, per call: fx_mstcn_params.fused_layers): conv GEMM (K = 3F)
// -> row-local epilogue -> 1x1 GEMM; both weight matrices in the packed fragment order of
// launch_pack_frag (FN x K floats each)
bool frl_supported(int F, const void* x, long long ldx, long long ld_other);
// whether rows / 32 row tiles cover FX_FRL_MIN_FILL (80) % of the CUs of the current device: below that the
// fused layer leaves too many CUs idle and the two tuned GEMMs are faster (T = 2048 x 2 videos, 50 %: 11.6-11.8
// vs 12.0 ms per step; the shipped yaml's 4096 + 2900 rows, 86 %: the fused layer 0.5 ms faster)
bool frl_fills_device(long long rows);
long long frl_packed_floats(int K);
// one matrix [FN][K] (leading dim ld) -> fragment order at dst (frl_packed_floats(K) floats)
struct FragJob {
  const float* src;
  float* dst;
  int ld, K;
};
constexpr int FRAG_JOBS = 48;   // matrices per pack launch
int launch_pack_frag(const FragJob* jobs, int n, hipStream_t s);
int launch_frl(const float* x, long long ldx, int M, int T, int dil, int dir, const int* seq_off, int nseq,
               const float* w1p, const float* bias1, int relu1, const float* resid1, long long ldr1, float* out1,
               long long ldo1, const float* w2p, const float* bias2, const float* resid2, long long ldr2,
               const float* gate2, long long ldg2, float* out2, long long ldo2, float drop_p,
               unsigned long long drop_seed, hipStream_t s, float vdrop_p = 0.f, unsigned long long vdrop_seed = 0,
               float* out3 = nullptr, long long ldo3 = 0);

}  // namespace fx
