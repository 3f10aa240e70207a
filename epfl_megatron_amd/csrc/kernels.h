// Host-side launcher declarations for the gfx950 kernels (implemented in *.hip).
// Pointers are device pointers; `dt` is an ema::DType; no launcher synchronises.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ema {

enum DType { DT_F32 = 0, DT_F16 = 1, DT_BF16 = 2 };

// ---- norms.hip ---------------------------------------------------------------
int norm_bwd_partials(int64_t rows);
int norm_bwd_workspace_rows(int64_t rows);  // rows of the fp32 [*, H] partial workspace
int norm_max_hidden(int dtype);
// res/sum_out (nullable): fused residual add, the norm input is x + res and
// is also written to sum_out.  dres (nullable): added to dx in backward.
// dw_acc / db_acc (nullable): the weight / bias gradients go into these fp32
// buffers (the parameters' main_grad; += when accumulate) instead of dw / db.
void rmsnorm_fwd(const void* x, const void* res, void* sum_out, const void* w, void* y,
                 float* rstd, int64_t rows, int H, float eps, int dt, hipStream_t s);
void rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd,
                 const void* dres, void* dx, float* dw_part, void* dw, float* dw_acc,
                 int accumulate, int64_t rows, int H, int dt, hipStream_t s);
void layernorm_fwd(const void* x, const void* res, void* sum_out, const void* w, const void* b,
                   void* y, float* mean, float* rstd, int64_t rows, int H, float eps, int dt,
                   hipStream_t s);
void layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean,
                   const float* rstd, const void* dres, void* dx, float* dw_part,
                   float* db_part, void* dw, void* db, float* dw_acc, float* db_acc,
                   int accumulate_w, int accumulate_b, int64_t rows, int H, int dt,
                   hipStream_t s);

// ---- rope.hip ----------------------------------------------------------------
// In-place rotation of q (r heads per group) and k (1 head per group) of a
// [s, b, ng, r+2, hd] tensor with element strides (ss, sb, sg, sh); k_only:
// the key heads only.
void rope_qkv_inplace(void* qkv, const float* cos, const float* sin, const int64_t* pos,
                      int64_t pos_stride_b, int S, int B, int G, int R, int HD, int64_t ss,
                      int64_t sb, int64_t sg, int64_t sh, int offset, int inverse, int k_only,
                      int dt, hipStream_t s);

// ---- activations.hip -----------------------------------------------------------
void glu_fwd(const void* x, void* y, int64_t rows, int F, int kind, int dt, hipStream_t s);
void glu_bwd(const void* dy, const void* x, void* dx, int64_t rows, int F, int kind, int dt,
             hipStream_t s);
void gelu_fwd(const void* x, const void* bias, void* y, int64_t rows, int F, int approx,
              int dt, hipStream_t s);
void gelu_bwd(const void* dy, const void* x, const void* bias, void* dx, int64_t rows, int F,
              int approx, int dt, hipStream_t s);

// ---- cross_entropy.hip -----------------------------------------------------------
void ce_fwd_fused(const void* logits, const int64_t* target, float* loss, float* lse,
                  int64_t rows, int V, int dt, hipStream_t s);
void ce_row_max(const void* logits, float* rmax, int64_t rows, int V, int dt, hipStream_t s);
void ce_sumexp_target(const void* logits, const int64_t* target, const float* rmax,
                      float* sumexp, float* tlogit, int64_t rows, int V, int64_t vstart, int dt,
                      hipStream_t s);
void ce_bwd(const void* logits, const int64_t* target, const float* lse, const float* dloss,
            void* dlogits, int64_t rows, int V, int64_t vstart, int dt, hipStream_t s);

// ---- softmax.hip -------------------------------------------------------------------
// x [B, NP, SQ, SK]; mask (mode 2) uint8/bool [B, 1, SQ, SK]; mode 0 none, 1 causal.
void softmax_fwd(const void* x, const uint8_t* mask, int64_t mask_bs, void* y, int64_t B,
                 int64_t NP, int SQ, int SK, float scale, int mode, int dt, hipStream_t s);
void softmax_bwd(const void* dy, const void* y, void* dx, int64_t rows, int SK, float scale,
                 int dt, hipStream_t s);

// ---- optim.hip ----------------------------------------------------------------------
void chunked_sumsq(const float* grad, const int64_t* table, int n_chunks, float* partial,
                   float* out, hipStream_t s);
struct AdamArgs {
  float lr[8];
  float wd[8];
  float beta1, beta2, eps, bc1, bc2, grad_scale;
  int adam_w_mode;
  // Optional device step state written by opt_prep (nullptr: use the host
  // scalars above): [0] grad scale (clip coef / loss scale), [1] skip flag
  // (non-finite grad norm), [2] step count (bias correction).
  const float* dev_state;
};
// One-thread epilogue of the grad-norm reduction: grad norm, clip coefficient,
// non-finite flag and step count, all on the device (no host sync per step).
// st = [scale, found_inf, step, grad_norm].
void opt_prep(const float* norm_sq, const float* inv_scale, float clip, float* st, hipStream_t s);
void flat_adam(float* master, void* model_out, int model_dt, const float* grad, float* m,
               float* v, const int64_t* table, int n_chunks, const AdamArgs& a, hipStream_t s);

// ---- dropout.hip --------------------------------------------------------------------------
// out = res + dropout(x [+ x2] [+ bias[col]]), Philox-4x32-10 keyed by (seed, offset);
// n % 8 == 0, h % 8 == 0 (bias length).  bwd: dx = dout * mask / (1 - p), mask regenerated.
void bias_dropout_add_fwd(const void* x, const void* x2, const void* bias, const void* res,
                          void* out, int64_t n, int64_t h, float p, uint64_t seed, uint64_t offset,
                          int dt, hipStream_t s);
void bias_dropout_add_bwd(const void* dout, void* dx, int64_t n, float p, uint64_t seed,
                          uint64_t offset, int dt, hipStream_t s);

// ---- flash_attn_fwd.hip / flash_attn_bwd.hip -------------------------------------------------
struct AttnParams {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  float* lse;  // [b, nq, sq]
  int b, sq, sk, nq, nkv, hd;
  // element strides; query head j at (j / r) * q_sg + (j % r) * q_sh, kv group g at g * k_sg.
  int64_t q_sb, q_ss, q_sg, q_sh;
  int64_t k_sb, k_ss, k_sg;
  int64_t v_sb, v_ss, v_sg;
  int64_t o_sb, o_ss, o_sh;  // o / dout share strides
  int causal;
  float scale;
  // Optional fused RoPE (interleaved pairs, fp32 tables [max_pos, hd/2]):
  // forward rotates Q in registers and writes it back in place (the block
  // that owns the rows); backward applies R^T to dQ and dK in its epilogues.
  const float* rope_cos;
  const float* rope_sin;
  const int64_t* rope_pos;  // [b, s] position ids (row stride rope_pos_sb) or null: row index
  int64_t rope_pos_sb;
  // Optional document (varlen) mask for packed sequences (--reset_attention_mask,
  // sq == sk): int32 [b, s] first position of the document holding each
  // position, and [b, s] one past its last position.  Key k is visible to
  // query q iff doc_start[q] <= k (<= q under the causal mask): the forward /
  // dQ kernels start each query block at its first document's first key tile,
  // the dK/dV kernel stops each key block at its last document's end.
  const int* doc_start;
  const int* doc_end;
  // Diagnostics only (null in production): per-workgroup s_memrealtime
  // stamps [entry, prologue done, loop done, exit, cu, xcc, 0, 0] (fa_set_stamps).
  unsigned long long* stamps;
  int64_t stamps_n;  // elements of the stamps buffer
  // lse element strides (batch, head); the row stride is 1
  int64_t lse_sb, lse_sh;
  // Forward only, context-parallel ring attention (parallel/context.py): a
  // running fp32 output o32 (element strides o32_sb / ss / sh, head_dim
  // contiguous) and the running lse.  merge = 0: store this pair's normalised
  // output and lse there; merge = 1: log-sum-exp combine them with what is
  // there.  p.o (16-bit) is not written when o32 is set.
  float* o32;
  int64_t o32_sb, o32_ss, o32_sh;
  int merge;
  // causal diagonal offset: key k is visible to query q iff k <= q + coff
  // (default sk - sq, bottom-right aligned; a context-parallel pair whose keys
  // all precede its queries passes sk: no causal cut, document starts only)
  int coff;
  // Set by the launchers (fa_pair_ncu): a causal forward / dQ grid of exactly
  // two blocks per CU, all resident at once, dispatched one block per CU and
  // then a second: blocks lin and lin + ncu share a CU, so the second round
  // runs the query blocks lightest-first (block lin >= ncu takes the place of
  // 3 ncu - 1 - lin in the heavy-first order) and every CU gets a heavy + a
  // light block.  0: plain heavy-first order.
  int pair_ncu;
};
// pair_ncu for a causal grid of `grid` blocks of `waves` waves (0: no pairing);
// fa_set_pairing(false) turns it off (tests: bitwise equal outputs either way)
int fa_pair_ncu(int causal, long grid, int waves, int hd);
void fa_set_pairing(bool on);
// the split-key forward for grids of at most one 4-wave block per CU (on by
// default; EMA_FA_KV2=0 / fa_set_kv2(false): the 4-wave forward)
void fa_set_kv2(bool on);
bool flash_attn_kv2(int b, int sq, int nq, int hd);  // that grid runs split-key
struct AttnBwdParams {
  AttnParams f;
  const void* dout;
  void* dq;  // same strides as q
  void* dk;  // same strides as k
  void* dv;  // same strides as v
  float* ndelta;  // fp32 [b, nq, sq]: -delta, written by the dQ kernel (initial dP accumulator)
  float* lse2;    // fp32 [b, nq, sq]: lse * log2(e), written by the dQ kernel
  float* dkv_ws;  // fp32 [kv_split][b][nkv][sk][2][hd] partial dK / dV (kv_split > 1)
  int kv_split;    // query heads of a KV group split over this many dK/dV workgroups
};
// How many workgroups share one KV group's query heads in the dK/dV kernel:
// the smallest divisor of r = nq / nkv that gives >= 512 workgroups (GQA/MQA
// with few KV heads per rank, e.g. Llama-2-70B or Falcon-40B under TP, would
// otherwise fill a quarter of the 256 CUs).  1 when nothing is gained.
inline int flash_attn_kv_split(int b, int sk, int nq, int nkv) {
  const int r = nq / nkv;
  const long base = (long)((sk + 127) / 128) * nkv * b;
  if (r <= 1 || base >= 512) return 1;
  for (int s = 2; s <= r; ++s)
    if (r % s == 0 && base * s >= 512) return s;
  return r;
}
// Waves per forward / dQ workgroup: 8 (256 query rows, one block per CU) on
// big grids, 4 (128 rows, two blocks per CU) at head_dim 64 and when the
// 8-wave grid would give fewer than two blocks per CU (few heads per TP rank):
// profiles/r2c_fa_waves_ab.txt.  EMA_FA_WAVES=4|8 overrides.
int flash_attn_waves(int b, int sq, int nq, int hd);
void flash_attn_fwd(const AttnParams& p, int dt, hipStream_t s);

// ---- flash_decode.hip: one query token per (batch, head) against a KV cache ----
struct DecodeParams {
  const void* q;  // query head j of group g at b*q_sb + g*q_sg + (j % r)*q_sh
  const void* k;  // key i of group g at b*k_sb + i*k_ss + g*k_sg
  const void* v;
  void* o;  // head `head` at b*o_sb + head*o_sh
  int b, sk, nq, nkv, hd;
  int64_t q_sb, q_sg, q_sh;
  int64_t k_sb, k_ss, k_sg;
  int64_t v_sb, v_ss, v_sg;
  int64_t o_sb, o_sh;
  float scale;
  float* ws_o;   // fp32 [b][nq][splits][hd] chunk partials
  float* ws_ml;  // fp32 [b][nq][splits][2] chunk (max, sum) in log2 units
  // optional device int32: the number of valid keys (<= sk).  The grid is
  // sized for sk (the cache capacity) and chunks past the length exit early,
  // so one launch serves every step of a captured hipGraph decode loop.
  const int* kv_len;
  // zeroed uint32 [flash_decode_counters()]: arrivals per (batch, head slice)
  // when a sequence is split over several workgroups; the last one to arrive
  // combines the chunk partials and re-arms its counter
  unsigned* counters;
  int kpw;  // keys per wave: 64 / 16 / 8 (flash_decode_kpw picks; chunk = 4 kpw keys)
};
int flash_decode_kpw(int b, int sk, int nq, int nkv);

// ---- decode_tail.hip -----------------------------------------------------------------------------
// Graphed greedy decode step tail: argmax of each row of logits [b, V] (row
// stride ld) -> tokens[b], history[b, *step_idx], pos[b] += 1; the last
// workgroup advances *step_idx, *slot and *kv_len (counter: zeroed uint32).
void greedy_tail(const void* logits, int64_t ld, int V, int b, int dt, int64_t* tokens,
                 int64_t* history, int64_t hist_ld, int64_t* step_idx, int64_t* pos, int64_t* slot,
                 int* kv_len, unsigned* counter, hipStream_t s);
int flash_decode_splits(int sk, int kpw);
int flash_decode_counters(int b, int nq, int nkv);
void flash_decode(const DecodeParams& p, int dt, hipStream_t s);
void flash_attn_bwd(const AttnBwdParams& p, int dt, hipStream_t s);

// ---- xgmi_allreduce.hip --------------------------------------------------------------------------
// One-shot all-reduce over IPC-mapped peer memory (small messages; see the file
// header).  create: allocate this rank's region and write its IPC handle
// (xgmi_handle_size() bytes) to handle_out; open: map the peers' handles
// ([world][handle] bytes); all_reduce: out = sum over ranks of in (in-place ok,
// nbytes a multiple of 16, <= cap), on stream s.
int64_t xgmi_create(int rank, int world, int64_t cap, void* handle_out);
int xgmi_handle_size();
void xgmi_open(int64_t id, const void* handles);
int64_t xgmi_capacity(int64_t id);
void xgmi_all_reduce(int64_t id, const void* in, void* out, int64_t nbytes, int dt, hipStream_t s);
// out [world * nbytes] = every rank's in [nbytes], rank-major (in: disjoint or one chunk of out)
void xgmi_all_gather(int64_t id, const void* in, void* out, int64_t nbytes, int dt, hipStream_t s);
int xgmi_error(int64_t id);
void xgmi_set_timeout(int64_t id, int64_t ms);
int64_t xgmi_get_timeout(int64_t id);
void* xgmi_error_word(int64_t id);  // device int32, nonzero after a timed-out wait
void xgmi_destroy(int64_t id);

// ---- gemm_wgrad.hip ------------------------------------------------------------------------------
// G[N,K] (+)= dY[M,N]^T X[M,K]; dY/X bf16|fp16 row-major, G fp32 row-major.
// Split-K plan of a shape: tiles [0, main_tiles) run unsplit, tiles
// [tail_lin0, tail_lin0 + tail_tiles) split over nsplit token ranges (fp32
// workspace of wgrad_workspace_floats() floats; none needed when nsplit == 1).
struct WgradPlan {
  int main_tiles, tail_lin0, tail_tiles, nsplit;
};
bool wgrad_supported(int64_t M, int64_t N, int64_t K);
void wgrad_set_variant(int v);  // 4: persistent 4-wave kernel (default), 8: 8-wave ping-pong
WgradPlan wgrad_plan(int64_t M, int64_t N, int64_t K);
int64_t wgrad_workspace_floats(int64_t M, int64_t N, int64_t K);
// Token (row) order of X relative to dY in a wgrad: logical token q of dY is
// X's physical row
//   ((q / rows) % n1) * s1 + ((q / rows) / n1) * s2 + q % rows   (rows == 0: q)
// i.e. a two-level permutation of rows-sized groups.  It pairs the SP
// pipeline's piece-major gathers ([piece][rank][R] rows) with natural-order
// ([rank][piece][R]) rows without a permutation copy (parallel/tensor/
// layers.py).  rows % 32 == 0 (a 32-token subtile never crosses a group).
struct TokMap {
  int rows = 0, n1 = 1;
  int64_t s1 = 0, s2 = 0;
};
void wgrad_gemm(const void* dy, const void* x, float* g, int64_t M, int64_t N, int64_t K,
                bool accumulate, int dt, hipStream_t s, float* ws = nullptr, TokMap xmap = {});
// ---- gemm_nt.hip: C[M,N] = A[M,K] B[N,K]^T (forward / dgrad), GLU epilogues --
void gemm_nt_set_variant(int v);  // 4 or 8 waves per workgroup
bool gemm_nt_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc);
// Row-group remap of an operand's rows (the chunked TP all-gather / reduce-
// scatter overlap): logical row q lives at physical row
//   (q / rows) * stride + offset + q % rows        (rows == 0: identity)
struct RowMap {
  int rows = 0;
  int64_t stride = 0, offset = 0;
};
void gemm_nt(const void* a, const void* b, void* c, int64_t M, int64_t N, int64_t K, int64_t lda,
             int64_t ldb, int64_t ldc, int dt, hipStream_t s, RowMap amap = {}, RowMap cmap = {},
             float* ws = nullptr);
// fp32 workspace (floats) gemm_nt splits K into for few-tile products (0: none)
int64_t gemm_nt_workspace_floats(int64_t M, int64_t N, int64_t K);
int gemm_nt_ksplit(int64_t M, int64_t N, int64_t K);  // K split the plain product runs with
// fc1 forward: b = W1 [2F, K]; writes pre [M, 2F] and y = x1 * act(x2) [M, F]
// (rows of both outputs through cmap)
void gemm_nt_glu(const void* a, const void* b, void* pre, void* y, int64_t M, int64_t F,
                 int64_t K, int64_t lda, int64_t ldb, int kind, int dt, hipStream_t s,
                 RowMap cmap = {});
// fc2 dgrad: b = W2^T [F, K]; reads pre [M, 2F], writes d(pre) [M, 2F]
void gemm_nt_dglu(const void* a, const void* b, const void* pre, void* dpre, int64_t M, int64_t F,
                  int64_t K, int64_t lda, int64_t ldb, int kind, int dt, hipStream_t s);
bool flash_attn_supported(int hd, int dt);

// ---- skinny_gemm.hip: Y[M, N] = X[M, K] W[N, K]^T for decode batches (M <= 16) ----
bool skinny_gemm_supported(int64_t M, int64_t N, int64_t K);
void skinny_gemm(const void* x, const void* w, void* y, int64_t M, int64_t N, int64_t K, int dt,
                 hipStream_t s);
// Fused decode forms (skinny_gemm.hip header): epi 0 plain, 1 residual add,
// 2 GLU (N = F, W [2F, K]), 3 GQA QKV with rotary + KV-cache write.
struct SkinnyArgs {
  const void* x;        // [M, K]
  const void* w;        // [N, K] (GLU: [2N, K])
  void* y;              // [M, ldy]: output (QKV: the q heads, [M, nq * hd])
  int M, N, K;
  int64_t ldy;
  const void* norm_w;   // RMSNorm weight [K] (nullptr: no norm prologue)
  float eps;
  const void* res;      // EPI_RES: residual [M, ldr]
  int64_t ldr;
  int act;              // EPI_GLU: activation kind (0 swiglu, 1 geglu, 2 reglu, 3 liglu)
  // EPI_QKV
  int r, hd;            // q heads per KV group, head dim (features: [ng, r + 2, hd])
  const float* cos;     // rotary tables [max_pos, hd / 2]
  const float* sin;
  const int64_t* pos;   // absolute position of token m at pos[m * pos_sb]
  int64_t pos_sb;
  void* kcache;         // cache slot rows: cache + slot * c_ss + m * c_sb + g * hd
  void* vcache;
  int64_t c_ss, c_sb;
  const int64_t* slot_ptr;  // device slot index (graph decode) or nullptr: `slot`
  int64_t slot;
  int packed;           // 1: w is in the decode-packed layout (skinny_pack, K % 256 == 0)
};
void skinny_gemm_ex(const SkinnyArgs& p, int epi, int dt, hipStream_t s);
int skinny_glu_half_tail(int64_t F, int64_t K, bool norm, int64_t M);

// ---- transpose.hip -------------------------------------------------------------------------------
// dst[cols, rows] = src[rows, cols]^T for 16-bit elements; rows, cols multiples of 64.
bool transpose16_supported(int64_t rows, int64_t cols);
void transpose16(const void* src, void* dst, int64_t rows, int64_t cols, hipStream_t s);

}  // namespace ema
