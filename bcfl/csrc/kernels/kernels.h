// Host launchers of the bcfl gfx950 kernels (raw pointers + hipStream_t; no torch headers, so
// the .hip translation units compile fast and bindings.cpp owns all tensor plumbing).
// Every launcher returns 0 on success, <0 for an unsupported shape (the binding raises).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bcfl {

enum DType { DT_F32 = 0, DT_BF16 = 1 };

// ---- layernorm.hip ----------------------------------------------------------------------------
int bwd_blocks(int T);
int launch_bdaln_fwd(const void* y, const void* bias, const void* res, const void* gamma,
                     const void* beta, void* out, void* z, float* mean, float* rstd, int T, int H,
                     float eps, uint32_t p8, uint32_t ka, uint32_t kb, int dt, hipStream_t s);
int launch_bdaln_bwd(const void* dout, const void* z, const float* mean, const float* rstd,
                     const void* gamma, void* dz, void* dy, float* partial, int nblk, int T, int H,
                     uint32_t p8, uint32_t ka, uint32_t kb, int want_dbias, int dt, hipStream_t s,
                     int drop_in = 0);
// dst[keys[i]] = sum of src[perm[j]] over the run of equal sorted keys starting at i (no atomics,
// deterministic); piece: fp32 [T, H] scratch
int launch_segment_rowsum(const void* src, int src_dt, const int64_t* keys, const int64_t* perm,
                          float* piece, void* dst, int dst_dt, int T, int H, hipStream_t s);
int launch_segment_rowsum_i32(const void* src, int src_dt, const int* keys, const int* perm,
                              float* piece, void* dst, int dst_dt, int T, int H, hipStream_t s);
int launch_colsum(const float* partial, int nblk, int nk_stride, int k, int H, void* out, int dt,
                  hipStream_t s);
// reduce planes 0..2 of partial[nblk][3][H] into out0..2 (nullptr = skip) in one launch
int launch_colsum3(const float* partial, int nblk, int H, void* out0, void* out1, void* out2,
                   int dt0, int dt1, int dt2, hipStream_t s);
int launch_emb_ln_fwd(const int* ids, const int* pos, const int* tt, const void* word,
                      const void* posw, const void* typew, const void* gamma, const void* beta,
                      void* out, void* z, float* mean, float* rstd, int T, int H, float eps,
                      uint32_t p8, uint32_t ka, uint32_t kb, int dt, hipStream_t s);
int launch_rmsnorm_fwd(const void* x, const void* w, void* out, float* rstd, int T, int H,
                       float eps, int dt, hipStream_t s);
int launch_rmsnorm_bwd(const void* dout, const void* x, const void* w, const float* rstd, void* dx,
                       float* partial, int nblk, int T, int H, int dt, hipStream_t s);

// ---- elementwise.hip -----------------------------------------------------------------------------
// ---- xent.hip: classifier cross-entropy ------------------------------------------------------
int launch_xent_fwd(const void* logits, const int* labels, int B, int C, float* loss, void* grad,
                    int dt, hipStream_t s);
int launch_xent_stats(const void* logits, const int* labels, int B, int C, double* acc4, int dt,
                      hipStream_t s);
int launch_drop_mask(void* m, int dt, int64_t n, uint32_t p8, uint32_t ka, uint32_t kb,
                     hipStream_t s);
int launch_bias_act_fwd(const void* y, const void* bias, void* out, int64_t rows, int N, int act,
                        int dt, hipStream_t s);
int launch_bias_act_bwd(const void* dout, const void* y, const void* bias, void* dy,
                        float* partial, int nblk_rows, int64_t rows, int N, int act, int dt,
                        hipStream_t s);
int launch_swiglu_fwd(const void* gu, void* out, int64_t rows, int I, int dt, hipStream_t s);
int launch_swiglu_bwd(const void* dout, const void* gu, void* dgu, int64_t rows, int I, int dt,
                      hipStream_t s);
int launch_rope(const void* x, void* out, const int* pos, const float* cos, const float* sin,
                int64_t rows, int row_stride, int nrot, int d, int inverse, int dt, hipStream_t s);
int launch_cast_copy(void* dst, int dst_dt, const void* src, int src_dt, int64_t n, hipStream_t s);
int launch_axpby(float* y, const void* x, int x_dt, float a, float b, int64_t n, hipStream_t s);
int launch_delta_round_end(float* y, const float* x, float* cum, const float* d, float* cv,
                           void* wire, int wire_dt, void* param_out, int param_dt, float inv_l,
                           float scale, int64_t n, hipStream_t s);
int launch_mix(float* master, const void* const* nbrs, const int* nbr_dt, const float* w, int nn,
               float self_w, void* param_out, int param_dt, int64_t n, hipStream_t s);
int launch_delta_encode(const float* x, float* ref, void* out, int out_dt, int64_t n,
                        hipStream_t s);
int launch_adamw(float* master, const void* grad, int grad_dt, float* m, float* v,
                 void* param_out, int param_dt, float lr, float b1, float b2, float eps, float wd,
                 int step, int mode, float grad_scale, int64_t n, hipStream_t s);
int launch_adamw_mt(float* master, float* m, float* v, void* param_out, int param_dt,
                    const void* const* grads, const int64_t* offs, const int64_t* numels,
                    int ntens, int grad_dt, float lr, float b1, float b2, float eps, float wd,
                    int step, int mode, float grad_scale, const float* corr, float corr_lr,
                    hipStream_t s, const void* const* grads2 = nullptr,
                    const float* gscale = nullptr);
int64_t sumsq_mt_blocks(const int64_t* numels, int ntens);
int launch_clip_coef_mt(const void* const* grads, const void* const* grads2, const int64_t* numels,
                        int ntens, int grad_dt, float* partial, float max_norm, float* out,
                        hipStream_t s);
int launch_update_stats(const void* a, const void* b, int dt, int64_t n, int dim, uint32_t ka,
                        uint32_t kb, float* out, hipStream_t s);
int launch_block_sketch(const void* x, int x_dt, int64_t n, int dim, uint32_t ka, uint32_t kb,
                        float* out, hipStream_t s);

// ---- sha256.hip ------------------------------------------------------------------------------------
int launch_sha256_leaves(const uint8_t* data, int64_t nbytes, int64_t leaf_bytes, uint8_t* out,
                         int64_t nleaves, hipStream_t s);
// reduces [n, 32] digests to one root in place-ish using scratch (same size); returns ptr to root
int launch_sha256_merkle(uint8_t* level, uint8_t* scratch, int64_t n, uint8_t* root, hipStream_t s);

// ---- gemm.hip ----------------------------------------------------------------------------------
struct WgradParams {
  const void* G;   // [M, N] bf16, row stride ldg (grad of the layer output)
  const void* X;   // [M, K] bf16, row stride ldx (layer input)
  float* part;     // [S, N, K] fp32 split partials (S > 1)
  void* out;       // [N, K] bf16, row stride ldo
  int64_t ldg, ldx, ldo;
  int M, N, K, S, Mc;
  float* dbias_part = nullptr;  // [S, N] fp32 partial bias gradients (nullptr: no bias)
  void* dbias = nullptr;        // [N] bf16 bias gradient
};
// number of splits S and rows per split Mc for an M x N x K weight gradient (-1: unsupported)
int wgrad_splits(int M, int N, int K, int* Mc);
int launch_wgrad(const WgradParams& p, hipStream_t s);
// out[n, k] = bf16(sum_s part[s, n, k]); with bpart: dbias[n] = bf16(sum_s bpart[s, n])
int launch_wgrad_reduce(const float* part, int S, int N, int K, void* out, int64_t ldo,
                        const float* bpart, void* dbias, hipStream_t s, int SB = 0);
int wgrad_g8_bias_parts(int S);  // rows of the bias-partial buffer the g8 weight gradient needs
// weight gradient on the 8-phase kernel (gemm8.hip, both operands transposed-read): split count
// for an M x N x K problem (0 = shape not supported) and the launch (p.S / p.Mc from it)
int wgrad_g8_splits(int M, int N, int K, int* Mc, int slots_override = 0);  // slots: 0 = default
void set_g8_block_rows(int bm);   // 128 / 256 pins the block rows of auto-tiled g8 launches, 0 = auto
void set_g8_persistent(bool on);  // persistent BM=128 g8 grids (BCFL_G8_PERSIST overrides)
void set_wgrad_slots(int slots);  // weight-gradient tile slots, 0 = 64 (BCFL_G8_WGRAD_SLOTS overrides)
int launch_wgrad_g8(const WgradParams& p, hipStream_t s);

// ---- skinny.hip: tall-skinny LoRA products (HBM-bound) ---------------------------------------
struct SkinnyParams {
  const void* X;   // the big operand [M, K] (xwt) / [M, N] (ptx), bf16, row stride ldx
  int64_t ldx;
  const void* W;   // the skinny operand: [R, K] (xwt) / [M, R] (ptx), bf16, row stride ldw
  int64_t ldw;
  int M, N, K, R;  // R <= 64
  int S, kc;       // slices and reduction elements per slice (from skinny_*_splits)
  float* part;     // fp32 [S, M, 16 ceil(R/16)] (xwt) / [S, 16 ceil(R/16), N] (ptx)
  void* out;       // bf16 [M, Cz] (xwt, columns >= R zero) / [R, N] (ptx), row stride ldo
  int64_t ldo;
  int Cz;
  float scale;
  // ptx only, LoRA dB mode (bdr > 0): out is [N, bdr] with out[n, j] = scale * (W^T X)[blk(n) bdr
  // + j, n], blk(n) the block with boff[b] <= n < boff[b + 1] — the diagonal blocks of the stacked
  // product, transposed: out[boff[b]:boff[b + 1]] IS adapter b's B gradient (contiguous rows)
  int bdr = 0, nblk = 0;
  int boff[5] = {0, 0, 0, 0, 0};
};
int skinny_xwt_splits(int M, int K, int* kc);
int launch_skinny_xwt(const SkinnyParams& p, hipStream_t s);   // out = scale X W^T (+ zero cols)
int skinny_ptx_splits(int M, int N, int* mc);
int launch_skinny_ptx(const SkinnyParams& p, hipStream_t s);   // out = scale W^T X
// LoRA adapter packing: bb[N, k2] = s Bbd zero-padded (block b of r columns holds B_b [o_b, r] at
// rows boff[b]..), bbt[nr, N] = bb[:, :nr]^T (the operand of the backward's g (s Bbd) product)
struct LoraPackParams {
  const void* B[4];
  int boff[5];
  int nblk, r, N, k2;
  float s;
  void* bb;
  void* bbt;
};
int launch_lora_pack_b(const LoraPackParams& p, hipStream_t s);

// ---- linear.hip: dense-layer GEMMs with fused epilogues ------------------------------------------
// RESID: C = A B (+ tail) + aux (residual). SWIGLU (gate|up forward, ROW B = [gate; up] with the
// up block `pair` rows below the gate block): aux[M, 2 pair] = the bf16 projection [gate | up],
// C[M, pair] = silu(gate) * up. SWIGLU_BWD (down-projection dgrad, C = dgu [M, 2 pair]): with
// dA = A B (+ tail) and aux = [gate | up], C[:, n] = dA up silu'(gate), C[:, pair + n] = dA silu(gate).
enum LinearEpi { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_ACT = 2, EPI_DACT = 3, EPI_ACCUM = 4,
                 EPI_PARTIAL = 5, EPI_RESID = 6, EPI_SWIGLU = 7, EPI_SWIGLU_BWD = 8 };
struct LinearParams {
  const void* A;       // [M, K] bf16, row stride lda
  const void* B;       // NT: [N, K] (ldb);  NN: [K, N] (ldb)
  void* C;             // [M, N] bf16, row stride ldc
  int64_t lda, ldb, ldc;
  int M, N, K;
  int epi = EPI_STORE;
  int act = 0;                   // activation id (act.h) for EPI_BIAS_ACT / EPI_DACT
  const void* bias = nullptr;    // [N] bf16 (EPI_BIAS / EPI_BIAS_ACT)
  void* aux = nullptr;           // [M, N] bf16 pre-activation: written by EPI_BIAS_ACT, read by EPI_DACT
  int64_t ldaux = 0;
  int tile = -1;                 // -1 auto | 0: 128 x 128 (4 waves) | 1: 256 x 256 (8 waves)
};
int launch_linear_nt(const LinearParams& p, hipStream_t s);  // C = A B^T
int launch_linear_nn(const LinearParams& p, hipStream_t s);  // C = A B

// ---- gemm8.hip: 8-phase LDS-DMA MFMA GEMM (fwd / dgrad / wgrad layouts) --------------------
// C[M, N] = sum_k A(m, k) B(k, n). a_col: A(m, k) = A[k * lda + m] (else A[m * lda + k]);
// b_col: B(k, n) = B[k * ldb + n] (else B[n * ldb + k]). Split-K: `splits` slices of `kc` reduction
// elements each (EPI_PARTIAL writes fp32 part[split][M][ldc]).
struct G8Params {
  const void* A;
  const void* B;
  void* C;
  int64_t lda, ldb, ldc;
  int M, N, K;
  int a_col = 0, b_col = 0;
  int bm = 0;                    // block rows: 256 or 128 (block cols are always 256); 0 = auto
  int epi = EPI_STORE;
  int act = 0;
  const void* bias = nullptr;    // [N] bf16
  void* aux = nullptr;           // [M, N] bf16 (EPI_BIAS_ACT writes, EPI_DACT reads)
  int64_t ldaux = 0;
  // A COL (weight gradient, A = G^T) only: row sums of A over each split's K range, i.e. the bias
  // gradient sum_rows G, by MFMA against a ones operand in the n-tile-0 workgroups:
  // rowsum[(2 split + h) * M + m], h = the two k-halves of every K-tile (summed by the reduce)
  float* rowsum = nullptr;
  float* part = nullptr;         // EPI_PARTIAL: fp32 [splits, M, ldc]
  int splits = 1;
  int kc = 0;                    // reduction elements per split (multiple of 128 for ROW operands)
  // optional tail segment of the reduction (splits == 1, ROW A, EPI_STORE): C = A B + A2 B2 with
  // A2 / B2 of the same kinds as A / B and K2 (a multiple of 128) more reduction elements. ROW
  // tails are zero-padded to K2 columns; a COL B2 has K2rows valid k-rows (the rest read as 0).
  const void* A2 = nullptr;
  const void* B2 = nullptr;
  int64_t lda2 = 0, ldb2 = 0;
  int K2 = 0, K2rows = 0;
  int pair = 0;                  // EPI_SWIGLU / EPI_SWIGLU_BWD: the intermediate size I
};
int g8_supported(const G8Params& p);  // 0 = launchable
int g8_auto_bm(int M, int N, int splits);
int launch_g8(const G8Params& p, hipStream_t s);

// ---- attention.hip -----------------------------------------------------------------------------
struct AttnParams {
  const void* qkv;     // [T, (nh + 2 nkv) * d] bf16
  void* out;           // [T, nh * d] bf16
  float* lse;          // [T, nh] (natural log, of scale * q.k)
  const int* cu;       // [B + 1]
  int B, T, nh, nkv, d, max_s;
  float scale;
  int causal;
  uint32_t p8, ka, kb;
  uint32_t* mask = nullptr;  // dropout keep bitmask [T * nh * mask_w], WRITTEN here (if p8)
  int mask_w = 0;            // words per (token, head) row (attn_dropmask_words)
  // work order (attn_schedule): n_units entries (b << 12) | 128-row block, longest first; null =
  // every (b, block < ceil(max_s / 128)) in batch order
  const int* sched = nullptr;
  int n_units = 0;
};
struct AttnBwdParams {
  const void* qkv;
  const void* out;
  const void* dout;    // [T, nh * d]
  const float* lse;    // [T, nh]
  float* delta;        // [2, T, nh] scratch: the prepped row constants (lse, rowsum(dO * O))
  void* dqkv;          // [T, (nh + 2 nkv) * d]
  const int* cu;
  int B, T, nh, nkv, d, max_s;
  float scale;
  int causal;
  uint32_t p8, ka, kb;
  const uint32_t* mask = nullptr;
  int mask_w = 0;
  const int* sched_q = nullptr;  // query-block order (dq), as AttnParams::sched
  const int* sched_k = nullptr;  // key-block order (dk / dv)
  int n_units = 0;
};
// dropout keep bitmask, 1 bit per score: word (t * nh + h) * W + kw holds the 32 keys
// 32 kw + j; key j = 8 g + 4 c + e (g, e < 4, c < 2) is bit 8 e + g + 4 c (attn_mbit), the order
// in which the forward's MFMA layout produces the decisions. Written by the forward, read by the
// backward kernels.
int attn_dropmask_words(int max_s);  // W
int launch_attn_fwd(const AttnParams& p, hipStream_t s);

// ---- subset_attention.hip: one pooled query row per sequence vs all its keys ------------------
struct SubsetAttnParams {
  const void* qkv;   // [T, (nh + 2 nkv) * d] bf16
  void* out;         // [B, nh * d] bf16
  float* lse;        // [B, nh]
  const int* cu;     // [B + 1]
  const int* rows;   // [B] absolute token index of each sequence's pooled row
  int B, nh, nkv, d, max_s;
  float scale;
  int causal;
  uint32_t p8, ka, kb;
};
struct SubsetAttnBwdParams {
  const void* qkv;
  const void* out;
  const void* dout;  // [B, nh * d]
  const float* lse;
  void* dqkv;        // [T, (nh + 2 nkv) * d], zero-filled by the caller
  const int* cu;
  const int* rows;
  int B, nh, nkv, d, max_s;
  float scale;
  int causal;
  uint32_t p8, ka, kb;
};
int launch_subset_attn_fwd(const SubsetAttnParams& p, hipStream_t s);
int launch_subset_attn_bwd(const SubsetAttnBwdParams& p, hipStream_t s);
int launch_attn_bwd(const AttnBwdParams& p, hipStream_t s);

}  // namespace bcfl
