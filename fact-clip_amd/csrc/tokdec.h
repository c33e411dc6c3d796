// The persistent token-side decoder kernel's program (tokdec.hip): a few phases, by value in the
// kernel arguments, run by one launch with a grid barrier between them.  Built by decoder.cpp.
#pragma once

#include <cstddef>

#include <hip/hip_runtime.h>

namespace fx {

constexpr int TOK_MAXK = 768;    // K of a GEMM phase (its 32-row A tile is staged whole in LDS)
constexpr int TOK_MAXSA = 256;   // d_model of a self-attention item (head dim 32 x heads)
constexpr int TOK_MAXPH = 8;     // phases per launch

enum TokOp { TOK_GEMM = 0, TOK_SAFWD = 1, TOK_MHABWD = 2, TOK_LNROWS = 3 };
// how a phase's A rows are staged: as stored; LayerNorm forward of them (the stored rows are the
// pre-LN sum); LayerNorm backward (the stored rows are dL/d(LN output); staged: dR, dropout-masked)
enum TokAMode { TOK_A_PLAIN = 0, TOK_A_LN = 1, TOK_A_LNBWD = 2 };

struct TokLN {
  const float* w;              // gamma (LN / LNBWD)
  const float* b;              // beta (LN)
  float eps;
  // forward write duty (row-major (M, K)): LN output, x-hat, 1/std per row, output + pos
  float* y;
  float* xh;
  float* rs;
  const float* pos;
  float* y2;
  // backward inputs / outputs: x-hat, 1/std; dR (un-masked residual-path gradient), dU (masked)
  const float* xhat;
  const float* rstd;
  float* dr;
  float* du;
  unsigned drop_thr;           // dU = dR * keep (index m K + k), 0 = off
  float drop_scale;
  unsigned long long drop_seed;
};

struct TokPhase {
  int op, amode;
  int M, N, K, Kp;             // rows, output columns, depth, depth rounded up to 32
  const float* a;              // A rows (pre-LN sum for A_LN, dL/dy for A_LNBWD, dO for MHABWD)
  long long lda;
  const float* apos;           // staged A + apos (output columns < apos_ncols; SAFWD: q and k)
  long long ldpos;
  int apos_ncols;
  const float* w;              // B: W (N x K) row-major (y = x W^T), or with btrans W (K x N) (dx = dy W)
  long long ldw;
  int btrans;
  const float* bias;
  int relu;                    // 1: ReLU last, 2: ReLU before the dropout
  float alpha;
  unsigned drop_thr;           // epilogue dropout, index m N + n
  float drop_scale;
  unsigned long long drop_seed;
  const float* resid;
  long long ldr;
  const float* gate;           // out = 0 where gate <= 0
  long long ldg;
  float* c;
  long long ldc;
  TokLN ln;
  // attention items (SAFWD / MHABWD): nvid videos of Qv tokens, nh heads of 32, K = nh * 32
  int nvid, Qv, nh;
  float scale;
  float* qkv;                  // (M, 3K) saved q | k | v (SAFWD writes, MHABWD reads)
  float* probs;                // (nvid, nh, Qv, Qv) saved softmax
  unsigned attn_thr;
  float attn_scale;
  unsigned long long attn_seed;
};

struct TokProgram {
  TokPhase ph[TOK_MAXPH];
  int nphase, G;
  unsigned long long* bar;     // set by launch_tok
  unsigned* status;            // caller's status word (FX_STATUS_TOK_TIMEOUT)
  unsigned spin_max;
  int debug;                   // FX_TOK_DEBUG: count phase entries into status[1..2], synchronous launch
  unsigned long long* stamps;  // FX_TOK_DEBUG: s_memrealtime per (workgroup, phase): start, end of work
};

size_t tok_lds_bytes();
int launch_tok(TokProgram& prog, hipStream_t s);

}  // namespace fx
