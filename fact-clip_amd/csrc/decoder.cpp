// Action-token decoders, whole stack per call: SCADecoder (basic.py:525-557, SCALayer
// basic.py:454-523) and SADecoder (basic.py:561-593, SALayer basic.py:391-452).
//
// The reference runs each layer as ~15 ATen ops from Python (plus positional-encoding clones,
// autograd grad accumulations and MultiheadAttention's own reshapes).  Here one C call runs the
// whole decoder forward (or backward) on the caller's stream:
//   * the cross-attention key/value projections of ALL layers read the same frame memory, so
//     they are ONE GEMM  KV = memory . [Wk_0..Wk_{L-1} | Wv_0..Wv_{L-1}]^T  (T x 2AL) instead of
//     2L frame-level GEMMs; backward likewise folds into one dMemory GEMM (K = 2AL) and one
//     weight-gradient GEMM (the frame-level work of the decoder is three large GEMMs);
//   * the self-attention core over the Q tokens is one fused launch per direction
//     (attn_small.hip); the cross-attention core over T frames uses the MHA core GEMMs;
//   * residual adds ride in GEMM epilogues, bias gradients in the weight-gradient GEMMs.
// Post-norm, ReLU FFN, eval-mode dropout; SALayer/SCALayer value has no positional term
// (sa_value_w_pos = ca_value_w_pos = vpos = False, as the reference builds them).
#include <algorithm>
#include <cmath>
#include <vector>

#include "fx_common.h"
#include "ops.h"
#include "tokdec.h"

namespace fx {
namespace {

constexpr int MAXL = 16;
constexpr int kSmallTok = 64;   // tokens per video the fused small-MHA kernel holds in LDS

struct PackKV {
  const float* src[2 * MAXL];   // k_w[0..L-1], v_w[0..L-1]   (A x Hm each)
  const float* bsrc[2 * MAXL];  // in_proj_bias + A, + 2A       (A each)
  float* dst;                   // (2AL x Hm)
  float* bdst;                  // (2AL)
  int A, Hm, L;
};

// pack the per-layer cross-attention K/V weights and biases into one row-major (2AL x Hm) operand
__global__ void pack_kv_kernel(PackKV p) {
  const int blk = blockIdx.y;  // 0..2L-1
  const long long n = (long long)p.A * p.Hm;
  const float* src = p.src[blk];
  float* dst = p.dst + (long long)blk * n;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    dst[i] = src[i];
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < p.A; i += blockDim.x) p.bdst[blk * p.A + i] = p.bsrc[blk][i];
}

struct UnpackKV {
  float* dst[2 * MAXL];   // dk_w[l], dv_w[l]  (accumulate)
  float* bdst[2 * MAXL];  // d in_proj_bias + A, + 2A  (accumulate)
  const float* src;
  const float* bsrc;
  int A, Hm, L;
};

__global__ void unpack_kv_acc_kernel(UnpackKV p) {
  const int blk = blockIdx.y;
  const long long n = (long long)p.A * p.Hm;
  const float* src = p.src + (long long)blk * n;
  float* dst = p.dst[blk];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    dst[i] += src[i];
  if (blockIdx.x == 0 && p.bdst[blk])
    for (int i = threadIdx.x; i < p.A; i += blockDim.x) p.bdst[blk][i] += p.bsrc[blk * p.A + i];
}

// y = x . w^T + b + resid   (w (N, K) row stride ldw)
int linear_fwd_res(const float* x, long long ldx, int M, int K, const float* w, long long ldw, const float* b,
                   const float* resid, long long ldr, float* y, long long ldy, int N, hipStream_t s) {
  fx_gemm_desc d = gemm_desc(M, N, K, op_rows(x, ldx), op_rows(w, ldw), y, ldy);
  d.bias = b;
  d.resid = resid;
  d.ld_resid = ldr;
  return launch_gemm(d, s);
}

// dx = dy . w + resid   (w (N, K) row stride ldw)
fx_gemm_desc dx_res_desc(const float* dy, long long lddy, const float* w, long long ldw, int M, int K, int N,
                         const float* resid, long long ldr, float* dx, long long lddx, float* ws) {
  fx_gemm_desc d = gemm_desc(M, K, N, op_rows(dy, lddy), op_cols(w, ldw), dx, lddx);
  d.resid = resid;
  d.ld_resid = ldr;
  d.split_k = pick_split(M, K, N);
  d.workspace = ws;
  return d;
}

int linear_dx_res(const float* dy, long long lddy, const float* w, long long ldw, int M, int K, int N,
                  const float* resid, long long ldr, float* dx, long long lddx, float* ws, hipStream_t s) {
  fx_gemm_desc d = gemm_desc(M, K, N, op_rows(dy, lddy), op_cols(w, ldw), dx, lddx);
  d.resid = resid;
  d.ld_resid = ldr;
  d.split_k = pick_split(M, K, N);
  d.workspace = ws;
  return launch_gemm(d, s);
}

struct DecLayout {
  // per-layer saved offsets (relative to layer base) and the layer stride
  long long xq, qkv, psa, osa, xh1, rs1, t1, t1q, qc, pca, oca, xh2, rs2, t2, f1, xh3, rs3, t3, per_layer;
  long long layers, fxh, frs, fo, kv, mpos, total_saved;
  // workspace (fwd)
  long long wkv, bkv, wsp, total_ws_fwd;
  // workspace (bwd)
  long long dkv, dwkv, dbkv, dT, dS, dU, dF, dQKV, dO, dq, lnws, core, dmask, split, gdu, gdf, gdq, gdqkv,
      gdy, total_ws_bwd;
};

long long dec_split_ws(const fx_decoder_params* p, int R, int T) {
  const int A = p->A, FF = p->FF;
  long long sp = 0;
  sp = std::max(sp, dwdb_ws(R, A, 3 * A));
  sp = std::max(sp, dwdb_ws(R, A, 2 * A));   // q/k rows of the packed in-proj (value rows apart)
  sp = std::max(sp, dwdb_ws(R, A, A));
  sp = std::max(sp, dwdb_ws(R, A, FF));
  sp = std::max(sp, dwdb_ws(R, FF, A));
  sp = std::max(sp, split_ws(R, A, 3 * A));
  sp = std::max(sp, split_ws(R, A, FF));
  sp = std::max(sp, split_ws(R, FF, A));
  sp = std::max(sp, dwdb_ws(R, A, p->out_dim));
  sp = std::max(sp, split_ws(R, A, p->out_dim));
  if (p->cross) {
    const long long AL2 = 2LL * A * p->num_layers;
    sp = std::max(sp, split_ws(T, (int)AL2, p->Hm));
    sp = std::max(sp, dwdb_ws(T, p->Hm, (int)AL2));
    sp = std::max(sp, split_ws(T, p->Hm, (int)AL2));
    // key rows only (the memory-pos gradient and its dW piece): half the tiles, up to twice the split
    sp = std::max(sp, dwdb_ws(T, p->Hm, (int)(AL2 / 2)));
    // the K/V weight gradient on the side stream, split defer_split(T) ways
    sp = std::max(sp, (long long)defer_split(T) * AL2 * (p->Hm + 1));
    sp = std::max(sp, split_ws(T, p->Hm, (int)(AL2 / 2)));
  }
  return sp;
}

// frames of the longest video (ragged memory: mem_off; else T / nvid each)
int dec_tmax(const fx_decoder_params* p, int T, int nvid) {
  if (!p->cross) return 0;
  if (!p->mem_off) return T / nvid;
  int m = 0;
  for (int v = 0; v < nvid; ++v) m = std::max(m, p->mem_off[v + 1] - p->mem_off[v]);
  return m;
}

// the attention-core workspace: cross attention over the frames, self attention over > 64 tokens
long long dec_attn_ws(const fx_decoder_params* p, int nvid, int Qv, int Tv) {
  const int hd = p->A / p->nhead;
  long long w = p->cross ? tattn_ws_floats(nvid, Qv, Tv, hd, p->nhead) : 0;
  if (Qv > kSmallTok) w = std::max(w, tattn_ws_floats(nvid, Qv, Qv, hd, p->nhead));
  return w;
}

DecLayout dec_layout(const fx_decoder_params* p, int R, int T, int has_qpos, int has_mpos, int nvid) {
  DecLayout L{};
  const long long A = p->A, FF = p->FF, h = p->nhead, RA = (long long)R * A;
  const long long Qv = R / nvid, Tv = dec_tmax(p, T, nvid);   // tokens / frames (longest video) per video
  long long o = 0;
  L.xq = o; o += al64(has_qpos ? RA : 0);
  L.qkv = o; o += al64(3 * RA);
  L.psa = o; o += al64(nvid * h * Qv * Qv);
  L.osa = o; o += al64(RA);
  L.xh1 = o; o += al64(RA);
  L.rs1 = o; o += al64(R);
  L.t1 = o; o += al64(RA);
  if (p->cross) {
    L.t1q = o; o += al64(has_qpos ? RA : 0);
    L.qc = o; o += al64(RA);
    L.pca = o; o += al64(nvid * h * Qv);            // cross-attention log-sum-exp per (video, head, token)
    L.oca = o; o += al64(RA);
    L.xh2 = o; o += al64(RA);
    L.rs2 = o; o += al64(R);
    L.t2 = o; o += al64(RA);
  }
  L.f1 = o; o += al64((long long)R * FF);
  L.xh3 = o; o += al64(RA);
  L.rs3 = o; o += al64(R);
  L.t3 = o; o += al64(RA);
  L.per_layer = o;
  L.layers = 0;
  o = L.layers + L.per_layer * p->num_layers;
  L.fxh = o; o += al64(p->final_norm ? RA : 0);
  L.frs = o; o += al64(p->final_norm ? R : 0);
  L.fo = o; o += al64(p->final_norm ? RA : 0);
  const long long AL2 = 2 * A * p->num_layers;
  L.kv = o; o += al64(p->cross ? (long long)T * AL2 : 0);
  L.mpos = o; o += al64((p->cross && has_mpos) ? (long long)T * p->Hm : 0);
  L.total_saved = o;
  const long long sp = dec_split_ws(p, R, T);
  // forward workspace
  o = 0;
  L.wkv = o; o += al64(p->cross ? AL2 * p->Hm : 0);
  L.bkv = o; o += al64(p->cross ? AL2 : 0);
  const long long att = dec_attn_ws(p, nvid, (int)Qv, (int)Tv);
  L.wsp = o; o += al64(std::max(sp, att) + RA);
  L.total_ws_fwd = o;
  // backward workspace
  o = 0;
  L.dkv = o; o += al64(p->cross ? (long long)T * AL2 : 0);
  L.dwkv = o; o += al64(p->cross ? AL2 * p->Hm : 0);
  L.dbkv = o; o += al64(p->cross ? AL2 : 0);
  L.dT = o; o += al64(RA);
  L.dS = o; o += al64(RA);
  L.dU = o; o += al64(RA);
  L.dF = o; o += al64((long long)R * FF);
  L.dQKV = o; o += al64(3 * RA);
  L.dO = o; o += al64(RA);
  L.dq = o; o += al64(RA);
  L.lnws = o; o += al64(layernorm_bwd_ws_floats(R, (int)A));
  L.core = o; o += al64(att);
  L.dmask = o; o += al64((p->dropout > 0.f) ? RA : 0);   // masked branch gradient (training dropout)
  L.split = o; o += al64(sp);
  // every layer's output gradients of its token linears, kept for the weight-gradient GEMMs that run
  // after the chain (side stream): dU of the three LayerNorms, dF, dq, dQKV
  L.gdu = o; o += al64(3LL * p->num_layers * RA);
  L.gdf = o; o += al64((long long)p->num_layers * R * FF);
  L.gdq = o; o += al64((long long)p->num_layers * RA);
  L.gdqkv = o; o += al64(3LL * p->num_layers * RA);
  // every layer's three LayerNorm input gradients, kept for the batched LN weight / bias gradients
  // that follow the chain on the side stream (the chain's LN backward computes dx only)
  L.gdy = o; o += al64(3LL * p->num_layers * RA);
  L.total_ws_bwd = o;
  (void)FF;
  return L;
}

int dec_check(const fx_decoder_params* p, int R, int T, int nvid) {
  FX_REQUIRE(p && p->num_layers >= 1 && p->num_layers <= MAXL, "decoder: 1..16 layers");
  FX_REQUIRE(nvid >= 1 && nvid <= 32 && R % nvid == 0, "decoder: 1..32 videos, token rows split evenly");
  if (p->cross) {
    if (p->mem_off) {
      FX_REQUIRE(p->mem_off[0] == 0 && p->mem_off[nvid] == T, "decoder: memory offsets must span [0, T]");
      for (int v = 0; v < nvid; ++v) FX_REQUIRE(p->mem_off[v + 1] > p->mem_off[v], "decoder: empty video memory");
    } else {
      FX_REQUIRE(T % nvid == 0 && T >= nvid, "decoder: memory rows must split evenly over the videos");
    }
    FX_REQUIRE(p->Hm > 0, "decoder: cross attention needs memory rows");
  }
  R /= nvid;
  FX_REQUIRE(p->nhead > 0 && p->A % p->nhead == 0, "decoder: A must be divisible by nhead");
  FX_REQUIRE(R >= 1, "decoder: >= 1 token per video");
  FX_REQUIRE(p->A / p->nhead <= 64, "decoder: head dim must be <= 64");
  FX_REQUIRE(p->A <= 1024, "decoder: A <= 1024 (LayerNorm row kernel)");
  FX_REQUIRE(p->dropout >= 0.f && p->dropout < 1.f && p->attn_dropout >= 0.f && p->attn_dropout < 1.f,
             "decoder: dropout p in [0, 1)");
  return FX_OK;
}

// dropout site s of layer l (0 self-attn probs, 1 its residual branch, 2 cross-attn probs, 3 its residual
// branch, 4 FFN hidden, 5 FFN residual branch)
unsigned long long dec_seed(const fx_decoder_params* p, int l, int site) { return fx_drop_subseed(p->seed, 8 * l + site); }

// y = drop(x . w^T + b) + resid  (w (N, K) row stride ldw); p_drop 0: no mask
int linear_fwd_res_drop(const float* x, long long ldx, int M, int K, const float* w, long long ldw, const float* b,
                        const float* resid, long long ldr, float* y, long long ldy, int N, float p_drop,
                        unsigned long long seed, hipStream_t s) {
  fx_gemm_desc d = gemm_desc(M, N, K, op_rows(x, ldx), op_rows(w, ldw), y, ldy);
  d.bias = b;
  d.resid = resid;
  d.ld_resid = ldr;
  d.drop_p = p_drop;
  d.drop_seed = seed;
  return launch_gemm(d, s);
}


// ---------------------------------------------------------------- persistent token kernel (tokdec.hip)
// The token rows of the whole decoder as a few launches of tok_kernel: one program per stretch between
// two attention-over-T launches (forward: [ca-out, FFN1, FFN2] of layer l - 1 + [self-attention,
// sa-out, q-proj] of layer l; backward the same stretch reversed), every phase writing exactly the
// saved / workspace slots the separate-launch path writes, so the deferred weight-gradient GEMMs, the
// LayerNorm parameter gradients and the query-position gradient read the same buffers either way.
// Shapes it covers: <= 32 tokens per video, head dim 32, A <= 256, FF and out_dim <= 768 (the
// benchmark's SCADecoder / SADecoders); other decoders keep the separate launches.
bool dec_tok_ok(const fx_decoder_params* p, int R, int nvid, const void* const* ptrs, int nptr,
                const long long* lds, int nld) {
  if (!knobs().dec_tok) return false;
  const int Qv = R / nvid, A = p->A;
  bool ok = Qv >= 1 && Qv <= 32 && p->nhead * 32 == A && A <= TOK_MAXSA && p->FF % 32 == 0 && p->FF >= A &&
            p->FF <= TOK_MAXK && 3 * A <= TOK_MAXK && p->out_dim >= 4 && p->out_dim % 4 == 0 && p->out_dim <= TOK_MAXK;
  for (int i = 0; i < nptr && ok; ++i) ok = ptrs[i] == nullptr || ((uintptr_t)ptrs[i] & 15) == 0;
  // weights and LayerNorm parameters are read as float4 (a flat parameter buffer may misalign them)
  auto al = [](const void* q) { return q == nullptr || ((uintptr_t)q & 15) == 0; };
  for (int l = 0; l < p->num_layers && ok; ++l) {
    ok = al(p->sa_in_w[l]) && al(p->sa_out_w[l]) && al(p->ff1_w[l]) && al(p->ff2_w[l]) && al(p->ln_sa_w[l]) &&
         al(p->ln_sa_b[l]) && al(p->ln_ff_w[l]) && al(p->ln_ff_b[l]);
    if (ok && p->cross)
      ok = al(p->ca_q_w[l]) && al(p->ca_out_w[l]) && al(p->ln_ca_w[l]) && al(p->ln_ca_b[l]);
  }
  ok = ok && al(p->out_w) && (!p->final_norm || (al(p->fn_w) && al(p->fn_b)));
  for (int i = 0; i < nld && ok; ++i) ok = lds[i] % 4 == 0;
  return ok;
}

struct TokBuild {
  TokProgram prog{};
  hipStream_t s;
  int* status;
  explicit TokBuild(hipStream_t st, int* stat) : s(st), status(stat) {}
  static int items(const TokPhase& P) {
    if (P.op == TOK_SAFWD || P.op == TOK_MHABWD) return P.nvid * P.nh;
    if (P.op == TOK_LNROWS) return (P.M + 31) / 32;
    return ((P.M + 31) / 32) * ((P.N + 31) / 32);
  }
  int flush() {
    if (prog.nphase == 0) return FX_OK;
    int G = 1;
    for (int i = 0; i < prog.nphase; ++i) G = std::max(G, items(prog.ph[i]));
    prog.G = std::min(G, 256);
    prog.status = reinterpret_cast<unsigned*>(status);
    prog.spin_max = tok_spin_max();
    FX_REQUIRE(status, "decoder: the persistent token kernel needs the caller's status word (fx_decoder_params.status)");
    prof_begin(8, s);
    FX_TRY(launch_tok(prog, s));
    prof_end(8, s, 0.0, 0.0, 1);
    prog = TokProgram{};
    return FX_OK;
  }
  // a new phase (the program launches when full)
  TokPhase* add(int op, int amode, int M, int N, int K) {
    if (prog.nphase == TOK_MAXPH && flush() != FX_OK) return nullptr;
    TokPhase& P = prog.ph[prog.nphase++];
    P = TokPhase{};
    P.op = op;
    P.amode = amode;
    P.M = M;
    P.N = N;
    P.K = K;
    P.Kp = (K + 31) / 32 * 32;
    P.alpha = 1.f;
    return &P;
  }
};

void tok_drop(unsigned& thr, float& scale, unsigned long long& seed, float p, unsigned long long sd) {
  thr = p > 0.f ? std::max(fx_drop_thresh(p), 1u) : 0u;
  scale = 1.f / (1.f - p);
  seed = sd;
}

// y = x W^T (+ b) (+ relu) (+ dropout) (+ resid) into c
TokPhase* tok_gemm(TokBuild& tb, int amode, int M, int N, int K, const float* a, long long lda, const float* w,
                   long long ldw, int btrans, const float* bias, float* c, long long ldc) {
  TokPhase* P = tb.add(TOK_GEMM, amode, M, N, K);
  if (!P) return nullptr;
  P->a = a;
  P->lda = lda;
  P->w = w;
  P->ldw = ldw;
  P->btrans = btrans;
  P->bias = bias;
  P->c = c;
  P->ldc = ldc;
  return P;
}

int dec_fwd_tok(const fx_decoder_params* p, const float* tgt, long long ldt, int R, const float* qpos, int nvid,
                int Qv, int Tv, const float* kv, float* out, long long ldo, float* saved, const DecLayout& L,
                float* u, float* spl, hipStream_t s) {
  const int A = p->A, FF = p->FF, h = p->nhead, hd = A / h, NL = p->num_layers, AL2 = 2 * A * NL;
  const float eps = p->eps > 0.f ? p->eps : 1e-5f;
  const float pd = p->dropout, pa = p->attn_dropout;
  const float scale = 1.0f / std::sqrt((float)hd);
  TokBuild tb(s, p->status);
  auto blk = [&](int l) { return saved + L.layers + (long long)l * L.per_layer; };
  auto lnp = [&](TokPhase* P, const float* w, const float* b) {
    P->ln.w = w;
    P->ln.b = b;
    P->ln.eps = eps;
  };
  // self-attention of layer l from x (layer 0: tgt) or LN3(u) of layer l - 1, then sa-out -> u, then the
  // next operand: cross decoders q-proj (LN1(u) + qpos), else FFN of the SALayer (below)
  auto self_attn = [&](int l) -> int {
    float* b = blk(l);
    TokPhase* P = tb.add(TOK_SAFWD, l == 0 ? TOK_A_PLAIN : TOK_A_LN, R, 3 * A, A);
    FX_REQUIRE(P, "decoder: token program");
    if (l == 0) {
      P->a = tgt;
      P->lda = ldt;
      if (qpos) {   // the saved q / k input x + qpos of layer 0 (basic.py:438)
        P->ln.pos = qpos;
        P->ln.y2 = b + L.xq;
      }
    } else {
      float* pb = blk(l - 1);
      P->a = u;
      P->lda = A;
      lnp(P, p->ln_ff_w[l - 1], p->ln_ff_b[l - 1]);
      P->ln.y = pb + L.t3;
      P->ln.xh = pb + L.xh3;
      P->ln.rs = pb + L.rs3;
      if (qpos) {
        P->ln.pos = qpos;
        P->ln.y2 = b + L.xq;
      }
    }
    P->apos = qpos;
    P->ldpos = A;
    P->w = p->sa_in_w[l];
    P->ldw = A;
    P->bias = p->sa_in_b[l];
    P->c = b + L.osa;
    P->ldc = A;
    P->nvid = nvid;
    P->Qv = Qv;
    P->nh = h;
    P->scale = scale;
    P->qkv = b + L.qkv;
    P->probs = b + L.psa;
    tok_drop(P->attn_thr, P->attn_scale, P->attn_seed, pa, dec_seed(p, l, 0));
    // t1 (pre-LN) = x + dropout1(out_proj(o))
    const float* x = l == 0 ? tgt : blk(l - 1) + L.t3;
    const long long ldx = l == 0 ? ldt : A;
    P = tok_gemm(tb, TOK_A_PLAIN, R, A, A, b + L.osa, A, p->sa_out_w[l], A, 0, p->sa_out_b[l], u, A);
    FX_REQUIRE(P, "decoder: token program");
    P->resid = x;
    P->ldr = ldx;
    tok_drop(P->drop_thr, P->drop_scale, P->drop_seed, pd, dec_seed(p, l, 1));
    return FX_OK;
  };
  // FFN of layer l on LN(u) (LN2 for cross decoders, LN1 for SALayers): f1 = relu(W1 t + b1) -> u = t + W2 f1 + b2
  auto ffn = [&](int l) -> int {
    float* b = blk(l);
    const bool cr = p->cross != 0;
    TokPhase* P = tok_gemm(tb, TOK_A_LN, R, FF, A, u, A, p->ff1_w[l], A, 0, p->ff1_b[l], b + L.f1, FF);
    FX_REQUIRE(P, "decoder: token program");
    lnp(P, cr ? p->ln_ca_w[l] : p->ln_sa_w[l], cr ? p->ln_ca_b[l] : p->ln_sa_b[l]);
    P->ln.y = b + (cr ? L.t2 : L.t1);
    P->ln.xh = b + (cr ? L.xh2 : L.xh1);
    P->ln.rs = b + (cr ? L.rs2 : L.rs1);
    P->relu = pd > 0.f ? 2 : 1;
    tok_drop(P->drop_thr, P->drop_scale, P->drop_seed, pd, dec_seed(p, l, 4));
    P = tok_gemm(tb, TOK_A_PLAIN, R, A, FF, b + L.f1, FF, p->ff2_w[l], FF, 0, p->ff2_b[l], u, A);
    FX_REQUIRE(P, "decoder: token program");
    P->resid = b + (cr ? L.t2 : L.t1);
    P->ldr = A;
    tok_drop(P->drop_thr, P->drop_scale, P->drop_seed, pd, dec_seed(p, l, 5));
    return FX_OK;
  };
  for (int l = 0; l < NL; ++l) {
    float* b = blk(l);
    if (p->cross) {
      if (l > 0) {   // layer l - 1 after its attention over T: ca-out (+ t1) -> u, FFN
        float* pb = blk(l - 1);
        TokPhase* P = tok_gemm(tb, TOK_A_PLAIN, R, A, A, pb + L.oca, A, p->ca_out_w[l - 1], A, 0, p->ca_out_b[l - 1], u, A);
        FX_REQUIRE(P, "decoder: token program");
        P->resid = pb + L.t1;
        P->ldr = A;
        tok_drop(P->drop_thr, P->drop_scale, P->drop_seed, pd, dec_seed(p, l - 1, 3));
        FX_TRY(ffn(l - 1));
      }
      FX_TRY(self_attn(l));
      // q = (LN1(u) + qpos) W_q^T + b_q, with t1 / x-hat / rstd / t1 + qpos written
      TokPhase* P = tok_gemm(tb, TOK_A_LN, R, A, A, u, A, p->ca_q_w[l], A, 0, p->ca_in_b[l], b + L.qc, A);
      FX_REQUIRE(P, "decoder: token program");
      lnp(P, p->ln_sa_w[l], p->ln_sa_b[l]);
      P->ln.y = b + L.t1;
      P->ln.xh = b + L.xh1;
      P->ln.rs = b + L.rs1;
      if (qpos) {
        P->ln.pos = qpos;
        P->ln.y2 = b + L.t1q;
        P->apos = qpos;
        P->ldpos = A;
        P->apos_ncols = A;
      }
      FX_TRY(tb.flush());
      TAttnOpts o;
      o.koff = p->mem_off;
      o.drop_p = pa;
      o.drop_seed = dec_seed(p, l, 2);
      FX_TRY(launch_tattn_fwd(b + L.qc, A, kv + (long long)l * A, AL2, kv + (long long)(NL + l) * A, AL2, nvid, Qv, Tv,
                              hd, h, scale, b + L.oca, A, b + L.pca, spl, s, &o));
    } else {
      FX_TRY(self_attn(l));
      FX_TRY(ffn(l));
    }
  }
  float* lb = blk(NL - 1);
  if (p->cross) {
    TokPhase* P = tok_gemm(tb, TOK_A_PLAIN, R, A, A, lb + L.oca, A, p->ca_out_w[NL - 1], A, 0, p->ca_out_b[NL - 1], u, A);
    FX_REQUIRE(P, "decoder: token program");
    P->resid = lb + L.t1;
    P->ldr = A;
    tok_drop(P->drop_thr, P->drop_scale, P->drop_seed, pd, dec_seed(p, NL - 1, 3));
    FX_TRY(ffn(NL - 1));
  }
  // last LayerNorm (t3), the final norm, the output linear
  TokPhase* P = tb.add(TOK_LNROWS, TOK_A_LN, R, A, A);
  FX_REQUIRE(P, "decoder: token program");
  P->a = u;
  P->lda = A;
  lnp(P, p->ln_ff_w[NL - 1], p->ln_ff_b[NL - 1]);
  P->ln.y = lb + L.t3;
  P->ln.xh = lb + L.xh3;
  P->ln.rs = lb + L.rs3;
  const float* fin = lb + L.t3;
  if (p->final_norm) {
    P = tb.add(TOK_LNROWS, TOK_A_LN, R, A, A);
    FX_REQUIRE(P, "decoder: token program");
    P->a = lb + L.t3;
    P->lda = A;
    lnp(P, p->fn_w, p->fn_b);
    P->ln.y = saved + L.fo;
    P->ln.xh = saved + L.fxh;
    P->ln.rs = saved + L.frs;
    fin = saved + L.fo;
  }
  P = tok_gemm(tb, TOK_A_PLAIN, R, p->out_dim, A, fin, A, p->out_w, A, 0, p->out_b, out, ldo);
  FX_REQUIRE(P, "decoder: token program");
  return tb.flush();
}

// The backward chain (fx_decoder_bwd's separate-launch loop, same slots): per layer, the LN3 backward staged
// into the FFN2 dX product, FFN1 dX + residual, the LN2 backward staged into the ca-out dX product,
// (attention over T), dq W_q + residual, the LN1 backward staged into the sa-out dX product, the self-
// attention backward per (video, head), [dq | dk | dv] W_in + residual.
int dec_bwd_tok(const fx_decoder_params* p, int R, int nvid, int Qv, int Tv, const float* dout, long long lddo,
                float* dtgt, long long lddt, const float* saved, float* ws, const DecLayout& L, float* dkv,
                hipStream_t s) {
  const int A = p->A, FF = p->FF, h = p->nhead, hd = A / h, NL = p->num_layers, AL2 = 2 * A * NL;
  const long long RA = (long long)R * A;
  const float pd = p->dropout, pa = p->attn_dropout;
  const float scale = 1.0f / std::sqrt((float)hd);
  TokBuild tb(s, p->status);
  auto blk = [&](int l) { return saved + L.layers + (long long)l * L.per_layer; };
  auto dy_slot = [&](int k, int l) { return ws + L.gdy + ((long long)k * NL + l) * RA; };
  auto slot_u = [&](int k, int l) { return ws + L.gdu + ((long long)k * NL + l) * RA; };
  float* dO = ws + L.dO;
  float* dmask = ws + L.dmask;
  const float* xl = blk(NL - 1) + L.t3;
  (void)xl;
  // LN backward staged into a product: dR (un-masked, residual path) and dU (masked branch) written
  auto lnb = [&](TokPhase* P, const float* w, const float* xh, const float* rs, int k, int l, int site) {
    P->ln.w = w;
    P->ln.xhat = xh;
    P->ln.rstd = rs;
    P->ln.du = slot_u(k, l);
    P->ln.dr = pd > 0.f ? dmask : nullptr;
    tok_drop(P->ln.drop_thr, P->ln.drop_scale, P->ln.drop_seed, pd, dec_seed(p, l, site));
  };
  auto dres = [&](int k, int l) -> const float* { return pd > 0.f ? dmask : slot_u(k, l); };
  // top: dfin = dout W_out (+ the final norm's backward) -> dT of the last layer
  {
    float* dT = dy_slot(0, NL - 1);
    TokPhase* P = tok_gemm(tb, TOK_A_PLAIN, R, A, p->out_dim, dout, lddo, p->out_w, A, 1, nullptr,
                           p->final_norm ? ws + L.dS : dT, A);
    FX_REQUIRE(P, "decoder: token program");
    if (p->final_norm) {
      P = tb.add(TOK_LNROWS, TOK_A_LNBWD, R, A, A);
      FX_REQUIRE(P, "decoder: token program");
      P->a = ws + L.dS;
      P->lda = A;
      P->ln.w = p->fn_w;
      P->ln.xhat = saved + L.fxh;
      P->ln.rstd = saved + L.frs;
      P->ln.dr = dT;
    }
  }
  // FFN (+ its LN) of layer l: dF = (LNbwd(dT) masked) W2 * (f1 > 0) [/ (1 - p)]; dT2 = dR + dF W1
  auto ffn_bwd = [&](int l) -> int {
    const float* b = blk(l);
    const bool cr = p->cross != 0;
    float* dF = ws + L.gdf + (long long)l * R * FF;
    TokPhase* P = tok_gemm(tb, TOK_A_LNBWD, R, FF, A, dy_slot(0, l), A, p->ff2_w[l], FF, 1, nullptr, dF, FF);
    FX_REQUIRE(P, "decoder: token program");
    lnb(P, p->ln_ff_w[l], b + L.xh3, b + L.rs3, 0, l, 5);
    P->gate = b + L.f1;
    P->ldg = FF;
    if (pd > 0.f) P->alpha = 1.f / (1.f - pd);
    P = tok_gemm(tb, TOK_A_PLAIN, R, A, FF, dF, FF, p->ff1_w[l], A, 1, nullptr, dy_slot(cr ? 1 : 2, l), A);
    FX_REQUIRE(P, "decoder: token program");
    P->resid = dres(0, l);
    P->ldr = A;
    return FX_OK;
  };
  // self-attention (+ its LN) of layer l: dO = LNbwd1(dT1) W_o ; [dq|dk|dv] ; dX = dR1 + dQKV W_in
  auto sa_bwd = [&](int l) -> int {
    const float* b = blk(l);
    TokPhase* P = tok_gemm(tb, TOK_A_LNBWD, R, A, A, dy_slot(2, l), A, p->sa_out_w[l], A, 1, nullptr, dO, A);
    FX_REQUIRE(P, "decoder: token program");
    lnb(P, p->ln_sa_w[l], b + L.xh1, b + L.rs1, 2, l, 1);
    float* dQKV = ws + L.gdqkv + (long long)l * 3 * RA;
    P = tb.add(TOK_MHABWD, TOK_A_PLAIN, R, 3 * A, A);
    FX_REQUIRE(P, "decoder: token program");
    P->a = dO;
    P->lda = A;
    P->c = dQKV;
    P->ldc = 3 * A;
    P->nvid = nvid;
    P->Qv = Qv;
    P->nh = h;
    P->scale = scale;
    P->qkv = const_cast<float*>(b + L.qkv);
    P->probs = const_cast<float*>(b + L.psa);
    tok_drop(P->attn_thr, P->attn_scale, P->attn_seed, pa, dec_seed(p, l, 0));
    if (l > 0 || dtgt) {
      P = tok_gemm(tb, TOK_A_PLAIN, R, A, 3 * A, dQKV, 3 * A, p->sa_in_w[l], A, 1, nullptr, l > 0 ? dy_slot(0, l - 1) : dtgt,
                   l > 0 ? A : lddt);
      FX_REQUIRE(P, "decoder: token program");
      P->resid = dres(2, l);
      P->ldr = A;
    }
    return FX_OK;
  };
  for (int l = NL - 1; l >= 0; --l) {
    const float* b = blk(l);
    FX_TRY(ffn_bwd(l));
    if (p->cross) {
      TokPhase* P = tok_gemm(tb, TOK_A_LNBWD, R, A, A, dy_slot(1, l), A, p->ca_out_w[l], A, 1, nullptr, dO, A);
      FX_REQUIRE(P, "decoder: token program");
      lnb(P, p->ln_ca_w[l], b + L.xh2, b + L.rs2, 1, l, 3);
      FX_TRY(tb.flush());
      float* dq = ws + L.gdq + (long long)l * RA;
      const float* kv = saved + L.kv;
      TAttnOpts o;
      o.koff = p->mem_off;
      o.drop_p = pa;
      o.drop_seed = dec_seed(p, l, 2);
      FX_TRY(launch_tattn_bwd(b + L.qc, A, kv + (long long)l * A, AL2, kv + (long long)(NL + l) * A, AL2, b + L.oca, A,
                              dO, A, b + L.pca, nvid, Qv, Tv, hd, h, scale, dq, A, dkv + (long long)l * A, AL2,
                              dkv + (long long)(NL + l) * A, AL2, ws + L.core, s, &o));
      P = tok_gemm(tb, TOK_A_PLAIN, R, A, A, dq, A, p->ca_q_w[l], A, 1, nullptr, dy_slot(2, l), A);
      FX_REQUIRE(P, "decoder: token program");
      P->resid = dres(1, l);
      P->ldr = A;
    }
    FX_TRY(sa_bwd(l));
  }
  return tb.flush();
}

}  // namespace
}  // namespace fx

using namespace fx;

extern "C" {

int fx_tok_gemm(const float* a, long long lda, int M, int N, int K, int amode, const float* ln_w, const float* ln_b,
                const float* w, long long ldw, int btrans, const float* bias, const float* resid, long long ldr,
                float* c, long long ldc, int* status, void* stream) {
  FX_REQUIRE(a && w && c && M > 0 && N > 0 && (amode == TOK_A_PLAIN || (amode == TOK_A_LN && ln_w && ln_b)),
             "tok gemm: bad arguments");
  TokBuild tb((hipStream_t)stream, status);
  TokPhase* P = tok_gemm(tb, amode, M, N, K, a, lda, w, ldw, btrans, bias, c, ldc);
  FX_REQUIRE(P, "tok gemm: program");
  P->resid = resid;
  P->ldr = ldr;
  if (amode == TOK_A_LN) {
    P->ln.w = ln_w;
    P->ln.b = ln_b;
    P->ln.eps = 1e-5f;
  }
  return tb.flush();
}

long long fx_decoder_saved_floats(const fx_decoder_params* p, int R, int T, int nvid, int has_qpos, int has_mpos) {
  return dec_layout(p, R, T, has_qpos, has_mpos, std::max(nvid, 1)).total_saved;
}

long long fx_decoder_workspace_floats(const fx_decoder_params* p, int R, int T, int nvid, int has_qpos,
                                      int has_mpos) {
  const DecLayout L = dec_layout(p, R, T, has_qpos, has_mpos, std::max(nvid, 1));
  return std::max(L.total_ws_fwd, L.total_ws_bwd);
}

int fx_decoder_fwd(const fx_decoder_params* p, const float* tgt, long long ldt, int R, const float* qpos,
                   long long ldqp, const float* mem, long long ldm, int T, int nvid, const float* mpos, long long ldmp,
                   float* out, long long ldo, float* saved, float* workspace, void* stream) {
  FX_TRY(dec_check(p, R, T, nvid));
  const int Qv = R / nvid, Tv = dec_tmax(p, T, nvid);
  hipStream_t s = (hipStream_t)stream;
  const int A = p->A, FF = p->FF, h = p->nhead, hd = A / h, NL = p->num_layers;
  const long long RA = (long long)R * A;
  const float eps = p->eps > 0.f ? p->eps : 1e-5f;
  const float pd = p->dropout, pa = p->attn_dropout;
  const float scale = 1.0f / std::sqrt((float)hd);
  const DecLayout L = dec_layout(p, R, T, qpos != nullptr, mpos != nullptr, nvid);
  FX_REQUIRE(!qpos || ldqp == A, "decoder: query_pos must be dense (R, A)");
  float* spl = workspace + L.wsp;
  WsBound wb(spl, L.total_ws_fwd - L.wsp);
  const int AL2 = 2 * A * NL;
  float* kv = saved + L.kv;
  if (p->cross) {
    // K/V projections of every layer in one frame-level GEMM (keys see mem + pos, values mem)
    PackKV pk{};
    for (int l = 0; l < NL; ++l) {
      pk.src[l] = p->ca_k_w[l];
      pk.src[NL + l] = p->ca_v_w[l];
      pk.bsrc[l] = p->ca_in_b[l] + A;
      pk.bsrc[NL + l] = p->ca_in_b[l] + 2 * A;
    }
    pk.dst = workspace + L.wkv;
    pk.bdst = workspace + L.bkv;
    pk.A = A;
    pk.Hm = p->Hm;
    pk.L = NL;
    fx_launch(pack_kv_kernel, dim3(std::min(cdiv((long long)A * p->Hm, 256), 256), 2 * NL), dim3(256), 0, s,
                       pk);
    FX_CHECK_HIP(hipGetLastError());
    // (profiling kind 9: the frame-level GEMM(s); algorithmic bytes = mem rows, packed weights, K/V rows)
    prof_begin(9, s);
    if (!mpos) {
      FX_TRY(linear_fwd(mem, ldm, T, p->Hm, workspace + L.wkv, workspace + L.bkv, kv, AL2, AL2, 0, s));
      prof_end(9, s, 2.0 * T * AL2 * p->Hm, 4.0 * ((double)T * p->Hm + (double)AL2 * p->Hm + (double)T * AL2));
    } else {
      const int AL = A * NL;
      FX_TRY(linear_fwd(mem, ldm, T, p->Hm, workspace + L.wkv, workspace + L.bkv, kv, AL2, AL, 0, s, -1, mpos, ldmp,
                        p->Hm));
      FX_TRY(linear_fwd(mem, ldm, T, p->Hm, workspace + L.wkv + (long long)AL * p->Hm, workspace + L.bkv + AL,
                        kv + AL, AL2, AL, 0, s));
      prof_end(9, s, 2.0 * T * AL2 * p->Hm, 4.0 * (2.0 * T * p->Hm + (double)AL2 * p->Hm + (double)T * AL2), 2);
      // keep mem + pos for the key weight gradient
      FX_TRY(add2(mem, ldm, mpos, ldmp, T, p->Hm, saved + L.mpos, p->Hm, 0, s));
    }
  }
  {
    const void* ptrs[3] = {tgt, qpos, out};
    const long long lds_[2] = {ldt, ldo};
    if (dec_tok_ok(p, R, nvid, ptrs, 3, lds_, 2)) {
      float* u = spl + (std::max(L.total_ws_fwd - L.wsp, RA) - RA);
      return dec_fwd_tok(p, tgt, ldt, R, qpos, nvid, Qv, Tv, kv, out, ldo, saved, L, u, spl, s);
    }
  }
  const float* x = tgt;
  long long ldx = ldt;
  for (int l = 0; l < NL; ++l) {
    float* b = saved + L.layers + l * L.per_layer;
    // --- self-attention over the tokens: q = k = x + qpos, v = x  (basic.py:495-503 / 438-444)
    const float* xq = x;
    long long ldxq = ldx;
    if (qpos) {   // layers >= 1: written by the previous layer's last LayerNorm (y + pos output)
      if (l == 0) FX_TRY(add2(x, ldx, qpos, A, R, A, b + L.xq, A, 0, s));
      xq = b + L.xq;
      ldxq = A;
    }
    float* qkv = b + L.qkv;   // (R, 3A): [q | k | v]
    if (!qpos) {
      FX_TRY(linear_fwd(x, ldx, R, A, p->sa_in_w[l], p->sa_in_b[l], qkv, 3 * A, 3 * A, 0, s));
    } else {   // q, k from x + qpos and v from x: two products, one grouped launch
      fx_gemm_desc d2[2];
      d2[0] = gemm_desc(R, 2 * A, A, op_rows(xq, ldxq), op_rows(p->sa_in_w[l], A), qkv, 3 * A);
      d2[0].bias = p->sa_in_b[l];
      d2[1] = gemm_desc(R, A, A, op_rows(x, ldx), op_rows(p->sa_in_w[l] + 2LL * A * A, A), qkv + 2 * A, 3 * A);
      d2[1].bias = p->sa_in_b[l] + 2 * A;
      FX_TRY(launch_gemm_group(d2, 2, s));
    }
    if (Qv <= kSmallTok) {
      FX_TRY(launch_mha_small_fwd(qkv, 3 * A, qkv + A, 3 * A, qkv + 2 * A, 3 * A, Qv, Qv, hd, h, scale, b + L.psa,
                                  b + L.osa, A, s, nvid, pa, dec_seed(p, l, 0)));
    } else {   // more tokens than the LDS-resident kernel holds: the attention-over-T kernels, lse kept in psa
      TAttnOpts o;
      o.drop_p = pa;
      o.drop_seed = dec_seed(p, l, 0);
      FX_TRY(launch_tattn_fwd(qkv, 3 * A, qkv + A, 3 * A, qkv + 2 * A, 3 * A, nvid, Qv, Qv, hd, h, scale, b + L.osa, A,
                              b + L.psa, spl, s, &o));
    }
    // t1 = LN(x + dropout1(out_proj(o)))
    float* u = spl + (std::max(L.total_ws_fwd - L.wsp, RA) - RA);   // last RA floats of the scratch
    FX_TRY(linear_fwd_res_drop(b + L.osa, A, R, A, p->sa_out_w[l], A, p->sa_out_b[l], x, ldx, u, A, A, pd,
                               dec_seed(p, l, 1), s));
    // (cross-attention decoders with query positions: the LayerNorm also writes t1 + qpos, the query
    // operand below)
    const bool t1q = p->cross && qpos;
    FX_TRY(launch_layernorm_fwd_pos(u, A, nullptr, 0, p->ln_sa_w[l], p->ln_sa_b[l], eps, R, A, 0, b + L.t1, A,
                                    nullptr, b + L.rs1, b + L.xh1, A, t1q ? qpos : nullptr, A,
                                    t1q ? b + L.t1q : nullptr, A, s));
    const float* t2 = b + L.t1;
    if (p->cross) {
      // --- cross-attention onto the frames: q = t1 + qpos, k = mem + pos, v = mem (basic.py:504-515)
      const float* tq = t1q ? b + L.t1q : b + L.t1;
      FX_TRY(linear_fwd(tq, A, R, A, p->ca_q_w[l], p->ca_in_b[l], b + L.qc, A, A, 0, s));
      // every video's tokens over its own frames, all heads, one fused launch (attn_t.hip)
      TAttnOpts o;
      o.koff = p->mem_off;
      o.drop_p = pa;
      o.drop_seed = dec_seed(p, l, 2);
      FX_TRY(launch_tattn_fwd(b + L.qc, A, kv + (long long)l * A, AL2, kv + (long long)(NL + l) * A, AL2, nvid, Qv, Tv,
                              hd, h, scale, b + L.oca, A, b + L.pca, spl, s, &o));
      FX_TRY(linear_fwd_res_drop(b + L.oca, A, R, A, p->ca_out_w[l], A, p->ca_out_b[l], b + L.t1, A, u, A, A, pd,
                                 dec_seed(p, l, 3), s));
      FX_TRY(launch_layernorm_fwd(u, A, nullptr, 0, p->ln_ca_w[l], p->ln_ca_b[l], eps, R, A, 0, b + L.t2, A,
                                  nullptr, b + L.rs2, b + L.xh2, A, s));
      t2 = b + L.t2;
    }
    // --- FFN: t3 = LN(t2 + W2 relu(W1 t2 + b1) + b2)   (basic.py:516-522 / 446-450)
    if (pd > 0.f) {   // f1 = dropout(relu(W1 t2 + b1)) (the saved f1 is the dropped activation)
      fx_gemm_desc d = gemm_desc(R, FF, A, op_rows(t2, A), op_rows(p->ff1_w[l], A), b + L.f1, FF);
      d.bias = p->ff1_b[l];
      d.relu = 2;
      d.drop_p = pd;
      d.drop_seed = dec_seed(p, l, 4);
      FX_TRY(launch_gemm(d, s));
    } else {
      FX_TRY(linear_fwd(t2, A, R, A, p->ff1_w[l], p->ff1_b[l], b + L.f1, FF, FF, 1, s));
    }
    FX_TRY(linear_fwd_res_drop(b + L.f1, FF, R, FF, p->ff2_w[l], FF, p->ff2_b[l], t2, A, u, A, A, pd,
                               dec_seed(p, l, 5), s));
    // (the next layer's query operand t3 + qpos written beside t3)
    const bool nxq = qpos && l + 1 < NL;
    FX_TRY(launch_layernorm_fwd_pos(u, A, nullptr, 0, p->ln_ff_w[l], p->ln_ff_b[l], eps, R, A, 0, b + L.t3, A,
                                    nullptr, b + L.rs3, b + L.xh3, A, nxq ? qpos : nullptr, A,
                                    nxq ? b + L.per_layer + L.xq : nullptr, A, s));
    x = b + L.t3;
    ldx = A;
  }
  if (p->final_norm) {
    FX_TRY(launch_layernorm_fwd(x, ldx, nullptr, 0, p->fn_w, p->fn_b, eps, R, A, 0, saved + L.fo, A, nullptr,
                                saved + L.frs, saved + L.fxh, A, s));
    x = saved + L.fo;
    ldx = A;
  }
  return linear_fwd(x, ldx, R, A, p->out_w, p->out_b, out, ldo, p->out_dim, 0, s);
}

int fx_decoder_bwd(const fx_decoder_params* p, const fx_decoder_grads* g, const float* tgt, long long ldt, int R,
                   const float* qpos, const float* mem, long long ldm, int T, int nvid, const float* mpos,
                   long long ldmp, const float* dout, long long lddo, float* dtgt, long long lddt, float* dqpos,
                   float* dmem, long long lddm, float* dmpos, long long lddmp, const float* saved, float* workspace,
                   void* stream) {
  FX_TRY(dec_check(p, R, T, nvid));
  const int Qv = R / nvid, Tv = dec_tmax(p, T, nvid);
  hipStream_t s = (hipStream_t)stream;
  const int A = p->A, FF = p->FF, h = p->nhead, hd = A / h, NL = p->num_layers;
  const long long RA = (long long)R * A;
  const float scale = 1.0f / std::sqrt((float)hd);
  const float pd = p->dropout, pa = p->attn_dropout;
  const DecLayout L = dec_layout(p, R, T, qpos != nullptr, mpos != nullptr, nvid);
  const int AL2 = 2 * A * NL;
  float* ws = workspace;
  float* spl = ws + L.split;
  WsBound wb(spl, L.total_ws_bwd - L.split);
  float* lnws = ws + L.lnws;
  float* dT = ws + L.dT;     // gradient w.r.t. the current layer output
  float* dS = ws + L.dS;
  float* dO = ws + L.dO;
  float* dkv = ws + L.dkv;
  // out_linear and the final LayerNorm
  const float* xl = saved + L.layers + (NL - 1) * L.per_layer + L.t3;   // last layer output
  const float* fin = p->final_norm ? saved + L.fo : xl;
  // LN input gradient of layer l's LayerNorm k (0 FFN, 1 cross-attention, 2 self-attention): each
  // producer in the chain writes straight into the slot its consumer reads
  auto dy_slot = [&](int k, int l) { return ws + L.gdy + ((long long)k * NL + l) * RA; };
  const void* tptrs[3] = {dout, dtgt, qpos};
  const long long tlds[2] = {lddo, dtgt ? lddt : 4};
  const bool tok = dec_tok_ok(p, R, nvid, tptrs, 3, tlds, 2);
  if (tok) FX_TRY(dec_bwd_tok(p, R, nvid, Qv, Tv, dout, lddo, dtgt, lddt, saved, ws, L, dkv, s));
  dT = dy_slot(0, NL - 1);
  if (!tok) FX_TRY(linear_bwd_pair(desc_linear_dwdb(dout, lddo, fin, A, R, A, p->out_dim, g->out_w, g->out_b, 1, spl),
                         desc_linear_dx(dout, lddo, p->out_w, R, A, p->out_dim, p->final_norm ? dS : dT, A, 0, nullptr,
                                        0, spl),
                         s));
  if (p->final_norm && !tok)
    FX_TRY(launch_layernorm_bwd(dS, A, nullptr, 0, saved + L.fxh, A, p->fn_w, saved + L.frs, R, A, 0, dT, A, g->fn_w,
                                g->fn_b, lnws, s));
  // Weight gradients of the token linears: the chain below writes each layer's dU (three LayerNorm
  // outputs), dF, dq and dQKV into per-layer slots and computes only the input gradients; the dW/db
  // GEMMs of every layer follow the chain on the side stream, batched over the layers where the
  // gradient buffers are uniformly strided (~35 one-wave launches per step left the main stream).
  auto slot_u = [&](int k, int l) { return ws + L.gdu + ((long long)k * NL + l) * RA; };   // k: 0 ff, 1 ca, 2 sa
  for (int l = NL - 1; l >= 0 && !tok; --l) {
    const float* b = saved + L.layers + l * L.per_layer;
    dT = dy_slot(0, l);
    float* dU = slot_u(0, l);
    float* dF = ws + L.gdf + (long long)l * R * FF;
    float* dq = ws + L.gdq + (long long)l * RA;
    float* dQKV = ws + L.gdqkv + (long long)l * 3 * RA;
    // --- FFN + its LayerNorm:  dR = LN_bwd(dT) ; dU = dR * mask5 ; dF = (dU W2) * (f1 > 0) / (1 - p4) ;
    //     dT2 = dR + dF W1.  Without dropout dR and dU are the same buffer.
    float* dR = pd > 0.f ? ws + L.dmask : dU;   // residual-path gradient (un-masked)
    auto branch_mask = [&](float* du, int site) -> int {   // dU = dR * keep / (1 - p) of the site's mask
      if (pd <= 0.f) return FX_OK;
      return launch_dropout(dR, A, R, A, A, 0, pd, dec_seed(p, l, site), du, A, s);
    };
    FX_TRY(launch_layernorm_bwd(dT, A, nullptr, 0, b + L.xh3, A, p->ln_ff_w[l], b + L.rs3, R, A, 0, dR, A, nullptr,
                                nullptr, lnws, s));
    FX_TRY(branch_mask(dU, 5));
    {
      fx_gemm_desc d = desc_linear_dx(dU, A, p->ff2_w[l], R, FF, A, dF, FF, 0, b + L.f1, FF, spl);
      if (pd > 0.f) d.alpha = 1.f / (1.f - pd);   // f1 > 0 <=> kept and active: the gate is relu' * mask
      FX_TRY(launch_gemm(d, s));
    }
    dT = dy_slot(p->cross ? 1 : 2, l);
    FX_TRY(launch_gemm(dx_res_desc(dF, FF, p->ff1_w[l], A, R, A, FF, dR, A, dT, A, spl), s));   // dT2 = dR + dF W1
    if (p->cross) {
      // --- cross-attention + LN2
      dU = slot_u(1, l);
      if (pd <= 0.f) dR = dU;
      FX_TRY(launch_layernorm_bwd(dT, A, nullptr, 0, b + L.xh2, A, p->ln_ca_w[l], b + L.rs2, R, A, 0, dR, A, nullptr,
                                  nullptr, lnws, s));
      FX_TRY(branch_mask(dU, 3));
      FX_TRY(launch_gemm(desc_linear_dx(dU, A, p->ca_out_w[l], R, A, A, dO, A, 0, nullptr, 0, spl), s));
      const float* kv = saved + L.kv;
      TAttnOpts o;
      o.koff = p->mem_off;
      o.drop_p = pa;
      o.drop_seed = dec_seed(p, l, 2);
      FX_TRY(launch_tattn_bwd(b + L.qc, A, kv + (long long)l * A, AL2, kv + (long long)(NL + l) * A, AL2, b + L.oca, A,
                              dO, A, b + L.pca, nvid, Qv, Tv, hd, h, scale, dq, A, dkv + (long long)l * A, AL2,
                              dkv + (long long)(NL + l) * A, AL2, ws + L.core, s, &o));
      dT = dy_slot(2, l);
      // dT1 = dR + dq Wq (the query-position gradient's share, dq Wq again, follows the chain on the aux
      // stream)
      FX_TRY(launch_gemm(dx_res_desc(dq, A, p->ca_q_w[l], A, R, A, A, dR, A, dT, A, spl), s));
    }
    // --- self-attention + LN1
    dU = slot_u(2, l);
    if (pd <= 0.f) dR = dU;
    FX_TRY(launch_layernorm_bwd(dT, A, nullptr, 0, b + L.xh1, A, p->ln_sa_w[l], b + L.rs1, R, A, 0, dR, A, nullptr,
                                nullptr, lnws, s));
    FX_TRY(branch_mask(dU, 1));
    FX_TRY(launch_gemm(desc_linear_dx(dU, A, p->sa_out_w[l], R, A, A, dO, A, 0, nullptr, 0, spl), s));
    const float* qkv = b + L.qkv;
    if (Qv <= kSmallTok) {
      FX_TRY(launch_mha_small_bwd(qkv, 3 * A, qkv + A, 3 * A, qkv + 2 * A, 3 * A, b + L.psa, dO, A, Qv, Qv, hd, h,
                                  scale, dQKV, 3 * A, dQKV + A, 3 * A, dQKV + 2 * A, 3 * A, s, nvid, pa,
                                  dec_seed(p, l, 0)));
    } else {
      TAttnOpts o;
      o.drop_p = pa;
      o.drop_seed = dec_seed(p, l, 0);
      FX_TRY(launch_tattn_bwd(qkv, 3 * A, qkv + A, 3 * A, qkv + 2 * A, 3 * A, b + L.osa, A, dO, A, b + L.psa, nvid, Qv,
                              Qv, hd, h, scale, dQKV, 3 * A, dQKV + A, 3 * A, dQKV + 2 * A, 3 * A, ws + L.core, s, &o));
    }
    float* dX = l == 0 ? nullptr : dy_slot(0, l - 1);   // the next (earlier) layer's output gradient
    // dX = dR + [dq | dk | dv] W_in  (q and k see x + qpos: with query positions their share dq W_q + dk W_k
    // is also the position gradient's, accumulated on the aux stream below)
    if (l > 0 || dtgt)
      FX_TRY(launch_gemm(dx_res_desc(dQKV, 3 * A, p->sa_in_w[l], A, R, A, 3 * A, dR, A, l > 0 ? dX : dtgt,
                                     l > 0 ? A : lddt, spl), s));
  }
  // Query-position gradient dqpos = sum over layers of dq_ca W_q,ca + [dq | dk]_sa W_{q,k},sa (the chain
  // above computed these products inside its dX GEMMs): accumulating GEMMs over the per-layer dq / dQKV
  // slots on the aux stream, beside the rest of this backward; the caller's stream waits for them
  // before returning.  (Split 1: the aux stream must not touch `spl`.)
  hipStream_t sa = s;
  if (qpos && dqpos) {
    sa = aux_fork(s);
    bool first = !p->dqpos_accumulate;
    auto acc = [&](const float* dy, long long lddy, const float* w, int N) -> int {
      fx_gemm_desc d = desc_linear_dx(dy, lddy, w, R, A, N, dqpos, A, first ? 0 : 1, nullptr, 0, nullptr);
      d.split_k = 1;
      d.workspace = nullptr;
      first = false;
      return launch_gemm(d, sa);
    };
    for (int l = NL - 1; l >= 0; --l) {
      if (p->cross) FX_TRY(acc(ws + L.gdq + (long long)l * RA, A, p->ca_q_w[l], A));
      FX_TRY(acc(ws + L.gdqkv + (long long)l * 3 * RA, 3 * A, p->sa_in_w[l], 2 * A));
    }
  }
  hipStream_t sd = side_fork(s, 1);
  {
    // one weight-gradient kind over all layers: dW_l (+)= dy_l^T x_l (+ db_l), layer l's operands at layer
    // 0's plus l times a stride; batched when the parameter gradients are uniformly strided (views of
    // one flat buffer), else one launch per layer.  Split 1: the side stream must not touch `spl`,
    // which the main stream's remaining GEMMs use.  The products are collected and launched up to four
    // per grouped launch (launch_gemm_group: independent direct-kernel problems in one launch)
    std::vector<fx_gemm_desc> pend;
    auto kind = [&](int l0, int nl, const float* dy, long long lddy, long long dy_bs, const float* xx, long long ldxx,
                    long long x_bs, int K, int N, float* const* gw, float* const* gb, long long b_off,
                    long long w_off) -> int {
      if (nl <= 0) return FX_OK;
      bool uni = nl > 1;
      for (int l = l0; l < l0 + nl && uni; ++l)
        uni = gw[l] && (!gb || gb[l]) && gw[l] - gw[l0] == (long long)(l - l0) * (gw[l0 + 1] - gw[l0]) &&
              (!gb || gb[l] - gb[l0] == (long long)(l - l0) * (gb[l0 + 1] - gb[l0]));
      const int step = uni ? nl : 1;
      for (int l = l0; l < l0 + nl; l += step) {
        if (!gw[l]) continue;
        fx_gemm_desc d = desc_linear_dwdb(dy + (l - l0) * dy_bs, lddy, xx + (l - l0) * x_bs, ldxx, R, K, N,
                                          gw[l] + w_off, gb ? gb[l] + b_off : nullptr, 1, nullptr);
        d.split_k = 1;
        d.workspace = nullptr;
        if (step > 1) {
          d.batch = step;
          d.a.batch_stride = dy_bs;
          d.b.batch_stride = x_bs;
          d.c_batch_stride = gw[l0 + 1] - gw[l0];
          d.c_last_batch_stride = gb ? gb[l0 + 1] - gb[l0] : 0;
        }
        pend.push_back(d);
      }
      return FX_OK;
    };
    const long long PL = L.per_layer;
    const float* b0 = saved + L.layers;
    if (tok && (g->out_w || g->out_b)) {   // the output linear's weight gradient (the separate-launch path pairs it with its dX)
      fx_gemm_desc d = desc_linear_dwdb(dout, lddo, fin, A, R, A, p->out_dim, g->out_w, g->out_b, 1, nullptr);
      d.split_k = 1;
      d.workspace = nullptr;
      pend.push_back(d);
    }
    FX_TRY(kind(0, NL, slot_u(0, 0), A, RA, b0 + L.f1, FF, PL, FF, A, g->ff2_w, g->ff2_b, 0, 0));
    FX_TRY(kind(0, NL, ws + L.gdf, FF, (long long)R * FF, b0 + (p->cross ? L.t2 : L.t1), A, PL, A, FF, g->ff1_w,
                g->ff1_b, 0, 0));
    if (p->cross) {
      FX_TRY(kind(0, NL, slot_u(1, 0), A, RA, b0 + L.oca, A, PL, A, A, g->ca_out_w, g->ca_out_b, 0, 0));
      FX_TRY(kind(0, NL, ws + L.gdq, A, RA, b0 + (qpos ? L.t1q : L.t1), A, PL, A, A, g->ca_q_w, g->ca_in_b, 0, 0));
    }
    FX_TRY(kind(0, NL, slot_u(2, 0), A, RA, b0 + L.osa, A, PL, A, A, g->sa_out_w, g->sa_out_b, 0, 0));
    // self-attention in-projection: layer 0's input is tgt (its own pointer), layers >= 1 read the
    // previous layer's output from `saved`
    const float* dq0 = ws + L.gdqkv;
    if (!qpos) {
      FX_TRY(kind(0, 1, dq0, 3 * A, 3 * RA, tgt, ldt, 0, A, 3 * A, g->sa_in_w, g->sa_in_b, 0, 0));
      FX_TRY(kind(1, NL - 1, dq0 + 3 * RA, 3 * A, 3 * RA, b0 + L.t3, A, PL, A, 3 * A, g->sa_in_w, g->sa_in_b, 0, 0));
    } else {
      FX_TRY(kind(0, NL, dq0, 3 * A, 3 * RA, b0 + L.xq, A, PL, A, 2 * A, g->sa_in_w, g->sa_in_b, 0, 0));
      FX_TRY(kind(0, 1, dq0 + 2 * A, 3 * A, 3 * RA, tgt, ldt, 0, A, A, g->sa_in_w, g->sa_in_b, 2 * A, 2LL * A * A));
      FX_TRY(kind(1, NL - 1, dq0 + 3 * RA + 2 * A, 3 * A, 3 * RA, b0 + L.t3, A, PL, A, A, g->sa_in_w, g->sa_in_b,
                  2 * A, 2LL * A * A));
    }
    for (size_t i = 0; i < pend.size(); i += 4)   // 4: members per grouped launch (gemm_f32.hip GMAX)
      FX_TRY(launch_gemm_group(pend.data() + i, (int)std::min<size_t>(4, pend.size() - i), sd));
  }
  {
    // every layer's LayerNorm weight / bias gradients in one launch: dw += sum_rows dy * xhat, db += sum_rows dy
    // (the chain's LN backward computed dx only)
    LnGradJob jobs[3 * MAXL + 1];
    int nj = 0;
    if (tok && p->final_norm && (g->fn_w || g->fn_b)) jobs[nj++] = LnGradJob{dS, saved + L.fxh, g->fn_w, g->fn_b};
    for (int l = 0; l < NL; ++l) {
      const float* b = saved + L.layers + l * L.per_layer;
      auto add = [&](int k, long long xh_off, float* const* gw, float* const* gb) {
        if (!gw[l] && !gb[l]) return;
        jobs[nj++] = LnGradJob{dy_slot(k, l), b + xh_off, gw[l], gb[l]};
      };
      add(0, L.xh3, g->ln_ff_w, g->ln_ff_b);
      if (p->cross) add(1, L.xh2, g->ln_ca_w, g->ln_ca_b);
      add(2, L.xh1, g->ln_sa_w, g->ln_sa_b);
    }
    FX_TRY(launch_ln_param_grads(jobs, nj, R, A, A, A, sd));
  }
  if (p->cross) {
    // frame memory: dmem = dKV . Wkv ; dWkv = dKV^T [mem+pos | mem] ; dbkv = colsum(dKV)
    PackKV pk{};
    for (int l = 0; l < NL; ++l) {
      pk.src[l] = p->ca_k_w[l];
      pk.src[NL + l] = p->ca_v_w[l];
      pk.bsrc[l] = p->ca_in_b[l] + A;
      pk.bsrc[NL + l] = p->ca_in_b[l] + 2 * A;
    }
    float* wkv = ws + L.dwkv;   // packed weights first (for dmem), then reused for their gradient
    pk.dst = wkv;
    pk.bdst = ws + L.dbkv;
    pk.A = A;
    pk.Hm = p->Hm;
    pk.L = NL;
    const int AL = A * NL;
    if (dmem || dmpos) {
      fx_launch(pack_kv_kernel, dim3(std::min(cdiv((long long)A * p->Hm, 256), 256), 2 * NL), dim3(256), 0,
                         s, pk);
      FX_CHECK_HIP(hipGetLastError());
      if (dmem) FX_TRY(linear_dx(dkv, AL2, wkv, T, p->Hm, AL2, dmem, lddm, 0, nullptr, 0, spl, s));
      if (dmpos) FX_TRY(linear_dx(dkv, AL2, wkv, T, p->Hm, AL, dmpos, lddmp, 0, nullptr, 0, spl, s));
    }
    // dWkv = dKV^T [mem+pos | mem] and its unpacking into the parameter gradients depend on nothing
    // the rest of the backward needs: side stream (the frame-level GEMM, K = T rows, leaves the main
    // stream), split so each workgroup holds its CU for a short K range
    sd = side_fork(s, 2);
    const int ksp = sd != s ? defer_split(T) : 1;
    auto dw = [&](const float* a, const float* x, long long ldx_, int N, float* w, float* b) -> int {
      fx_gemm_desc d = desc_linear_dwdb(a, AL2, x, ldx_, T, p->Hm, N, w, b, 0, spl);
      d.split_k = std::max(d.split_k, ksp);
      return launch_gemm(d, sd);
    };
    if (!mpos) {
      FX_TRY(dw(dkv, mem, ldm, AL2, wkv, ws + L.dbkv));
    } else {
      FX_TRY(dw(dkv, saved + L.mpos, p->Hm, AL, wkv, ws + L.dbkv));
      FX_TRY(dw(dkv + AL, mem, ldm, AL, wkv + (long long)AL * p->Hm, ws + L.dbkv + AL));
    }
    UnpackKV uk{};
    for (int l = 0; l < NL; ++l) {
      uk.dst[l] = g->ca_k_w[l];
      uk.dst[NL + l] = g->ca_v_w[l];
      uk.bdst[l] = g->ca_in_b[l] ? g->ca_in_b[l] + A : nullptr;
      uk.bdst[NL + l] = g->ca_in_b[l] ? g->ca_in_b[l] + 2 * A : nullptr;
    }
    uk.src = wkv;
    uk.bsrc = ws + L.dbkv;
    uk.A = A;
    uk.Hm = p->Hm;
    uk.L = NL;
    fx_launch(unpack_kv_acc_kernel, dim3(std::min(cdiv((long long)A * p->Hm, 256), 256), 2 * NL), dim3(256),
                       0, sd, uk);
    FX_CHECK_HIP(hipGetLastError());
  }
  if (sd != s && !p->side_defer) FX_TRY(side_join_into(s));
  FX_TRY(aux_join_into(s, sa));
  return FX_OK;
}

}  // extern "C"
