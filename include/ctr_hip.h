/* C-ABI of libctrhip.so -- the MI355X (gfx950) kernels behind the CTRModel training hot path.
 *
 * The reference (biyotteu/toss-next-ctr-prediction) is pure PyTorch: it has no FFI.  Each entry
 * point below replaces the torch ops of one reference function, cited as path:line relative to the
 * reference root.  The Python host side (tossctr/_lib.py) binds these through ctypes; see
 * INTEGRATION.md for the binding a maintainer would add to the reference itself.
 *
 * Conventions (all entries):
 *   - device pointers are plain fp32 / int32 / uint32 arrays owned by the caller (PyTorch's caching
 *     allocator); the library never allocates on the hot path; scratch comes in via `ws` pointers
 *     sized by the matching *_ws_size query.
 *   - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream); no host sync inside.
 *   - return 0 on success, negative on error; ctr_last_error() returns a thread-local message.
 *   - dropout everywhere uses the counter-based mask {key, thresh16, scale} of csrc/common.h
 *     (spec shared with oracle/rng.py); thresh16 == 0 disables it.
 */
#ifndef CTR_HIP_H
#define CTR_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* ctr_last_error(void);
int ctr_abi_version(void);

/* ---------------------------------------------------------------------------------------------
 * Dense GEMM on fp32 MFMA (v_mfma_f32_16x16x4_f32):  C[M,N] = op(A)[M,K] * op(B)[K,N] (+ epilogue)
 * Replaces every nn.Linear / matmul on the path: MHA in/out projections (torch MHA via
 * src/models/dare.py:43,64), FFN (src/models/dare.py:45-48), QNN A=z@U (src/models/qnn_alpha.py:92),
 * MLP (src/models/qnn_alpha.py:78-84,129), fc head (src/models/wrapper.py:95-100) and their
 * backward dX / dW products.
 *   ta: A stored [K,M] (A^T row-major) instead of [M,K];  tb: B stored [N,K] instead of [K,N].
 *   splits > 1: K split across workgroups into ws (splits*M*N floats), reduced in fixed order.
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  const float* bias;     /* [N] added after the product (nullable)                                */
  const float* add;      /* [M,N] addend, row stride ld_add (nullable)                            */
  int ld_add;
  int act;               /* 0 none, 1 relu, 2 gelu(erf)                                           */
  float* pre;            /* store pre-activation (after bias/add), row stride ldc (nullable)      */
  int dact;              /* backward: 0 none, 1 relu'(aux), 2 gelu'(aux); multiplies the product   */
  const float* aux;      /* [M,N] pre-activation from the forward, row stride ldc                 */
  uint32_t drop_key, drop_thresh; /* dropout over linear index row*N+col (fwd: apply, bwd: mask)  */
  float drop_scale;
  const float* resid;    /* fused residual + RMSNorm over the whole row (requires N <= 64):       */
  int ld_resid;          /*   h = resid + (acc + bias); C = (w*h) * rsqrt(mean(h^2) + eps)        */
  const float* norm_w;   /*   src/models/dare.py:12-13, 64-70                                     */
  float* norm_h;         /*   saved h [M,N] (row stride ldc)                                      */
  float* norm_r;         /*   saved rsqrt factor [M]                                              */
  float norm_eps;
} ctr_gemm_epi_t;

/* Operand / result segments of one GEMM over concatenated buffers (ctr_gemm_seg): A columns k >= ka are
 * read from A2 (row stride lda2; A not transposed), B columns n >= nb from B2 (row stride ldb2; B not
 * transposed), C columns n >= nc are written to C2 (row stride ldc2; no row-indexed epilogue operand).
 * Null pointers disable a segment.  Used for the QNN MLP's first layer, whose input is [z | inter]
 * (src/models/qnn_alpha.py:120-124) -- one launch instead of two per product. */
typedef struct {
  const float* A2;
  int lda2, ka;
  const float* B2;
  int ldb2, nb;
  float* C2;
  int ldc2, nc;
} ctr_gemm_seg_t;

size_t ctr_gemm_ws_size(int M, int N, int splits);
int ctr_gemm(int M, int N, int K, const float* A, int lda, int ta, const float* B, int ldb, int tb,
             float* C, int ldc, const ctr_gemm_epi_t* epi, int splits, float* ws, void* stream);
int ctr_gemm_seg(int M, int N, int K, const float* A, int lda, int ta, const float* B, int ldb, int tb,
                 float* C, int ldc, const ctr_gemm_epi_t* epi, int splits, float* ws, const ctr_gemm_seg_t* seg,
                 void* stream);
/* ctr_gemm_seg with flags (seg nullable).  CTR_GEMM_BF16: the operands are rounded to bf16 (RNE) and
 * multiplied on v_mfma_f32_16x16x32_bf16 with fp32 accumulation -- the reference's
 * torch.autocast(bfloat16) matmul (src/train.py:133-139,158-164; amp: bf16); C and epilogues fp32.     */
#define CTR_GEMM_BF16 1
int ctr_gemm_ex(int M, int N, int K, const float* A, int lda, int ta, const float* B, int ldb, int tb,
                float* C, int ldc, const ctr_gemm_epi_t* epi, int splits, float* ws, const ctr_gemm_seg_t* seg,
                int flags, void* stream);
/* bf16-operand GEMM (amp: bf16 -- the reference's torch.autocast(bfloat16) nn.Linear of the QNN MLP,
 * src/models/qnn_alpha.py:120-124, src/train.py:133-139): A, B are bf16 images already in HBM (ta / tb as
 * in ctr_gemm: A (M, K) or stored (K, M); B (N, K) when tb, else (K, N)), fp32 accumulation on
 * v_mfma_f32_16x16x32_bf16, C and the epilogue fp32 (no fused RMSNorm; seg: the C2 result segment only).
 * ctr_gemm_bf16_ok: K % 64 == 0, leading dims % 8 == 0, M % 8 (ta) / N % 8 (!tb) == 0.
 * ctr_to_bf16: fp32 (rows, cols), row stride lds -> bf16 row stride ldd, round-to-nearest-even.     */
int ctr_gemm_bf16_ok(int M, int N, int K, int lda, int ta, int ldb, int tb, int splits);
int ctr_gemm_bf16(int M, int N, int K, const void* A, int lda, int ta, const void* B, int ldb, int tb,
                  float* C, int ldc, const ctr_gemm_epi_t* epi, int splits, float* ws, const ctr_gemm_seg_t* seg,
                  void* stream);
/* ctr_gemm_bf16 with flags.  CTR_GEMM_OUT_BF16: C (and the C2 segment) are bf16, the RNE of the fp32
 * accumulation (splits = 1) -- the dtype autocast gives the reference's matmul output, e.g. the QNN MLP's
 * input grad [dz | dinter] (src/models/qnn_alpha.py:120-124 under src/train.py:158-164).               */
#define CTR_GEMM_OUT_BF16 1
int ctr_gemm_bf16_ex(int M, int N, int K, const void* A, int lda, int ta, const void* B, int ldb, int tb,
                     void* C, int ldc, const ctr_gemm_epi_t* epi, int splits, float* ws, const ctr_gemm_seg_t* seg,
                     int flags, void* stream);
int ctr_to_bf16(const float* src, long lds, int rows, int cols, void* dst, long ldd, void* stream);
/* test / bench hook: the bf16 GEMM kernel form (0 automatic, 1 two-stage 128 x 128, 2 ring 256 x 128, 3 ring 128 x 128) */
void ctr_gemm_bf16_set_variant(int v);


/* Row-streaming GEMMs of the DARE encoder layer (MHA in_proj / out_proj, src/models/dare.py:53-62, and
 * their backward) for D in {16, 32}: M rows x a few-KB weight, HBM-bound           (rowgemm.hip)
 * C = A W^T (tb = 1, W (N, K)) or A W (tb = 0, W (K, N)); epilogue: + bias, + add, or the fused
 * residual + RMSNorm (h = resid + (acc + bias), C = norm_w h rsqrt(mean h^2 + eps), h / r saved).
 * Supported (K, N): (16,16) (16,48) (48,16) (32,32) (32,96) (96,32).                             */
int ctr_rowgemm_supported(int K, int N);
int ctr_rowgemm(int M, int K, int N, const float* A, int lda, const float* W, int tb, float* C, int ldc,
                const float* bias, const float* add, int ld_add, const float* resid, int ld_resid,
                const float* norm_w, float* norm_h, float* norm_r, float eps, void* stream);
/* weight + bias grad of one nn.Linear over M rows: slab row w (of ctr_rowgemm_wgrad_rows(M)) =
 * [dW (NO x NIN) | ... | db (NO) at o_db] partial over wave w's rows; ctr_colsum of the slab rows
 * (fixed order) lands them in the grad arena.  (NO, NIN): (16,16) (48,16) (32,32) (96,32).        */
int ctr_rowgemm_wgrad_rows(int M);
int ctr_rowgemm_wgrad(const float* dY, int ldy, const float* X, int ldx, int M, int NO, int NIN, float* slab,
                      long ld_slab, int o_db, void* stream);
/* amp: bf16 -- the in-projection's backward on the bf16 dqkv of ctr_attn_bwd_bf_oproj16 (uint16_t = bf16 bits,
 * widened exactly; W, X, the bias sums and the outputs fp32): ctr_rowgemm_a16 = ctr_rowgemm with a bf16 A,
 * (K, N) = (96, 32), epilogue + bias / + add; ctr_rowgemm_wgrad_y16 = ctr_rowgemm_wgrad with a bf16 dY,
 * (NO, NIN) = (96, 32).  Same bits as the fp32 forms on the widened values.                                  */
int ctr_rowgemm_a16(int M, int K, int N, const uint16_t* A, int lda, const float* W, int tb, float* C, int ldc,
                    const float* bias, const float* add, int ld_add, void* stream);
int ctr_rowgemm_wgrad_y16(const uint16_t* dY, int ldy, const float* X, int ldx, int M, int NO, int NIN, float* slab,
                          long ld_slab, int o_db, void* stream);
/* amp: bf16 forms of the two above for D = 64 (cfgs/v3_k148_s1.yaml; the reference's autocast F.linear,
 * src/train.py:158-168 over src/models/dare.py:53-62): operands rounded to bf16 (RNE), fp32 accumulation
 * and fp32 outputs, same arguments and epilogues.  (K, N): (64,64) (64,192) (192,64); wgrad (NO, NIN):
 * (64,64) (192,64), its slab rows counted by ctr_rowgemm_bf_wgrad_rows(M); db sums the fp32 dY.    (rowgemm_bf.hip) */
int ctr_rowgemm_bf_supported(int K, int N);
int ctr_rowgemm_bf(int M, int K, int N, const float* A, int lda, const float* W, int tb, float* C, int ldc,
                   const float* bias, const float* add, int ld_add, const float* resid, int ld_resid,
                   const float* norm_w, float* norm_h, float* norm_r, float eps, void* stream);
int ctr_rowgemm_bf_wgrad_rows(int M);
int ctr_rowgemm_bf_wgrad(const float* dY, int ldy, const float* X, int ldx, int M, int NO, int NIN, float* slab,
                         long ld_slab, int o_db, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Feature embeddings / context                                                    (embed.hip)
 * ------------------------------------------------------------------------------------------- */
/* NumericFeatureEmbedding / BinaryFeatureEmbedding.forward, src/models/feature_embed.py:19-27,42-48:
 * out[b, f*D + d] (row stride out_ld) = sum_k (x[b,f]*W[f,k] + bias[f,k]) * P[d,k]  (bias nullable) */
int ctr_feat_embed_fwd(const float* x, int B, int F, const float* W, const float* bias, const float* P, int fe,
                       int D, float* out, long out_ld, void* stream);
size_t ctr_feat_embed_bwd_ws(int B, int F, int D);
int ctr_feat_embed_bwd(const float* x, int B, int F, const float* W, const float* bias, const float* P, int fe, int D,
                       const float* dout, long dout_ld, float* dW, float* dbias, float* dP, float* ws, void* stream);
/* both groups (numeric, binary: src/models/wrapper.py:95-100 embeds both into the same rows) in one launch per
 * kernel: group 0's arguments then group 1's, as ctr_feat_embed_fwd / _bwd (each group its own ws); out / dout rows
 * share the stride.  Same sums, products and orders as two single-group calls.                                  */
int ctr_feat_embed_fwd2(const float* x0, int F0, const float* W0, const float* bias0, const float* P0, float* out0,
                        const float* x1, int F1, const float* W1, const float* bias1, const float* P1, float* out1, int B,
                        int fe, int D, long out_ld, void* stream);
int ctr_feat_embed_bwd2(const float* x0, int F0, const float* W0, const float* bias0, const float* P0,
                        const float* dout0, float* dW0, float* dbias0, float* dP0, float* ws0, const float* x1, int F1,
                        const float* W1, const float* bias1, const float* P1, const float* dout1, float* dW1,
                        float* dbias1, float* dP1, float* ws1, int B, int fe, int D, long dout_ld, void* stream);
/* CTRModel._embed_cats + emb_dropout, src/models/wrapper.py:106-112,149-150: hashed-bucket gather of
 * X_cat[b,c] from table c (tab_base + tab_off[c], row stride row_ld, or dims[c] when row_ld == 0;
 * tab_base NULL = arena) projected by P_c (arena + proj_off[c]).  Row-sharded tables pass the
 * batch's fetched rows as tab_base (tab_off 0, row_ld 64) and X_cat remapped to fetched-row ids.
 * cat_e = pre-dropout (B, Fc, D); xf (nullable) receives the dropped copy at row stride xf_ld.      */
int ctr_cat_embed_fwd(const int* xcat, int B, int Fc, const float* arena, const float* tab_base, const long* tab_off,
                      const long* proj_off, const int* dims, int row_ld, int D, float* cat_e, float* xf, long xf_ld,
                      uint32_t drop_key, uint32_t drop_thresh, float drop_scale, void* stream);
size_t ctr_cat_embed_bwd_ws(int B, int Fc);
/* backward: row-grad contributions (B*Fc rows x 64; columns k < d_c written, the rest left as they are --
 * pass a buffer zero-filled once, as its padding is never written) keyed row_base[c] + X_cat[b,c] for
 * ctr_rowgrad, and dP_c written into grad_arena + proj_goff[c].                                    */
int ctr_cat_embed_bwd(const int* xcat, int B, int Fc, const float* arena, const float* tab_base, const long* tab_off,
                      const long* proj_off, const int* dims, int row_ld, int D, const float* dcat,
                      const uint32_t* row_base, float* contrib,
                      uint32_t* keys, float* grad_arena, const long* proj_goff, float* ws, void* stream);
/* CTRModel._context_vector / _make_query, src/models/wrapper.py:114-136; mode 0 S1, 1 S2, 2 concat */
int ctr_context_fwd(const float* num_e, long num_ld, int Fn, const float* mask_e, long mask_ld, int Fm,
                    const float* cat_e, int Fc, int D, int B, int mode, int qi, const float* Wc, const float* bc,
                    float* ctx, float* hq, float* query, void* stream);
int ctr_context_bwd(const float* num_e, long num_ld, int Fn, const float* mask_e, long mask_ld, int Fm,
                    const float* cat_e, int Fc, int D, int B, int mode, int qi, const float* Wc, const float* hq,
                    const float* dquery, const float* dxf_cat, long dxf_ld, uint32_t drop_key, uint32_t drop_thresh,
                    float drop_scale, const float* dfc, long dfc_ld, float* dnum, float* dmask, float* dcat,
                    float* dpre, void* stream);

/* ---------------------------------------------------------------------------------------------
 * DARE                                                                            (dare.hip)
 * ------------------------------------------------------------------------------------------- */
/* DARE.topk_select, src/models/dare.py:116-138.  seq (B,L) int32 token ids; decay_log (L) =
 * log(exp(-(L-1-l)/max(1,tau)) + 1e-8); pads score -1e9; sorted top-K (ties: lower position first).
 * Outputs idx (B,K) positions, tok (B,K) token ids, vals (B,K), sel (B,K,D) = E_rep[tok].          */
int ctr_dare_topk_fwd(const int* seq, int B, int L, const float* q, const float* E_att, const float* E_rep, int D,
                      const float* decay_log, int K, int pad_id, int* idx, int* tok, float* vals, float* sel,
                      void* stream);
/* backward: dq (B,D); att row-grad contributions dvals*q (B*K, D) and keys (token or 0xFFFFFFFF for
 * pads, whose grads padding_idx drops); rep keys (the rep contributions are dsel itself).          */
int ctr_dare_topk_bwd(const int* tok, int B, int K, const float* q, const float* E_att, int D, const float* dvals,
                      int pad_id, float* dq, float* att_contrib, uint32_t* att_keys, uint32_t* rep_keys, void* stream);
/* DARE.forward gating/pool/aux head, src/models/dare.py:150-162; gating 0 softmax, 1 relu */
int ctr_pool_fwd(const float* x, const float* vals, int B, int K, int D, int gating, uint32_t drop_key,
                 uint32_t drop_thresh, float drop_scale, const float* waux, const float* baux, float* w, float* u,
                 float* xf_u, long xf_ld, float* aux, void* stream);
int ctr_pool_bwd(const float* x, const float* vals, const float* w, int B, int K, int D, int gating, uint32_t drop_key,
                 uint32_t drop_thresh, float drop_scale, const float* waux, const float* du, long du_ld,
                 const float* daux, float* dx, float* dvals, void* stream);
/* PositionalBias + head mean, src/models/dare.py:29-37,56-60: out[d] = mean_h rel[d,h] */
int ctr_pos_bias_mean(const float* rel, int H, int n, float* out, void* stream);
/* drel[d, h] = sum_p part[p, d] / H; part (the attention backward's diagonal partials) is scratch, reduced in place */
int ctr_pos_bias_grad(float* part, int nparts, int H, int n, float* drel, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Attention core of DAREEncoderLayer (MHA explicit path), src/models/dare.py:53-62    (attn.hip)
 * qkv (B*K, 3D) from the in-projection GEMM; o (B*K, D); mrow/lrow (B*H*K) row max / sum saved for
 * the recompute backward; drel_part (B*nparts, 2tk+1) positional-bias grad partials.
 * ------------------------------------------------------------------------------------------- */
int ctr_attn_mask_words(int B, int K, int H);   /* uint32 words of the dropout keep-bit mask */
void ctr_attn_set_generic(int on);   /* test hook: 1 = the unpacked forward even where the packed one applies */
/* mask (nullable without dropout): the forward stores the keep bits of p~, row ((b*H+h)*K + i),
 * ceil(K/32) words per row; the backward reads them instead of re-evaluating the hash.             */
int ctr_attn_fwd(const float* qkv, int B, int K, int H, int D, const float* relmean, int tk, float scale,
                 uint32_t drop_key, uint32_t drop_thresh, float drop_scale, uint32_t* mask, float* o, float* mrow,
                 float* lrow, void* stream);
int ctr_attn_bwd_nparts(int H, int K, int D);
int ctr_attn_bwd(const float* qkv, const float* o, const float* dO, int B, int K, int H, int D, const float* relmean,
                 int tk, float scale, uint32_t drop_key, uint32_t drop_thresh, float drop_scale, const uint32_t* mask,
                 const float* mrow, const float* lrow, float* dqkv, float* drel_part, void* stream);
/* amp: bf16 -- the same attention on bf16 MFMA (attn_mf.hip): products on bf16-rounded q*scale, k, v, dO, p~
 * and dS with fp32 accumulation, as the reference's autocast(bfloat16) baddbmm / bmm; softmax, dropout and dS
 * in fp32.  K <= 64 and head dim 4 or 8 (ctr_attn_bf_ok).  Arguments as ctr_attn_fwd / ctr_attn_bwd, except:
 * mask holds the keep bits in the kernels' lane layout (B*H x 2 x 64 words, <= ctr_attn_mask_words), mrow
 * the row max in log2 units -- both only meaningful to ctr_attn_bwd_bf; drel_part has B*ctr_attn_bwd_bf_nparts rows. */
int ctr_attn_bf_ok(int K, int H, int D);
int ctr_attn_fwd_bf(const float* qkv, int B, int K, int H, int D, const float* relmean, int tk, float scale,
                    uint32_t drop_key, uint32_t drop_thresh, float drop_scale, uint32_t* mask, float* o, float* mrow,
                    float* lrow, void* stream);
int ctr_attn_bwd_bf_nparts(int H);
int ctr_attn_bwd_bf(const float* qkv, const float* o, const float* dO, int B, int K, int H, int D,
                    const float* relmean, int tk, float scale, uint32_t drop_key, uint32_t drop_thresh,
                    float drop_scale, const uint32_t* mask, const float* mrow, const float* lrow, float* dqkv,
                    float* drel_part, void* stream);
/* amp: bf16 -- ctr_attn_bwd_bf with the out-projection's input grad fused in front (K <= 64, D = 32, 4 or 8 heads:
 * ctr_attn_bwd_bf_oproj_ok): dO = dh1 W_out (src/models/dare.py:53-62, MHA out_proj backward) is formed per workgroup
 * from the (B*K, 32) rows dh1 and out_proj.weight (32, 32) with the same bits as ctr_rowgemm(dh1, W_out, tb = 0), and
 * never written; the other arguments and outputs as ctr_attn_bwd_bf.                                          */
int ctr_attn_bwd_bf_oproj_ok(int K, int H, int D);
int ctr_attn_bwd_bf_oproj(const float* qkv, const float* o, const float* dh1, const float* w_out, int B, int K, int H,
                          int D, const float* relmean, int tk, float scale, uint32_t drop_key, uint32_t drop_thresh,
                          float drop_scale, const uint32_t* mask, const float* mrow, const float* lrow, float* dqkv,
                          float* drel_part, void* stream);
/* amp: bf16 -- the first half of an encoder layer in one launch, src/models/dare.py:53-62
 * (qkv = in_proj(x); o = attention(qkv); x1 = norm1(x + out_proj(o))): one workgroup per sample, K <= 64,
 * D = 32, 4 or 8 heads, tk <= 64 (ctr_attn_layer_fwd_ok).  Writes exactly what ctr_rowgemm (in_proj),
 * ctr_attn_fwd_bf and ctr_rowgemm (out_proj + residual + RMSNorm, eps) write -- qkv, o, mrow, lrow, mask, h1,
 * r1, x1 -- with the same bits (same summation orders).  rel_w = pbias.rel.weight ((2tk+1) x H) or null: the
 * head-mean bias is formed in the kernel and written to relmean (ctr_pos_bias_mean's bits) for the backward.   */
int ctr_attn_layer_fwd_ok(int K, int H, int D);
int ctr_attn_layer_fwd_bf(const float* x, int B, int K, int H, int D, const float* w_in, const float* b_in,
                          const float* rel_w, float* relmean, int tk, float scale, uint32_t drop_key, uint32_t drop_thresh,
                          float drop_scale, uint32_t* mask, const float* w_out, const float* b_out, const float* nw1,
                          float eps, float* qkv, float* o, float* mrow, float* lrow, float* h1, float* r1, float* x1,
                          void* stream);
/* amp: bf16 -- the saved projections in bf16 (uint16_t = bf16 bits).  ctr_attn_layer_fwd_bf16 writes qkv16 (B*K x 96)
 * = the operands the attention products take: bf16(q * scale) | bf16(k) | bf16(v) (RNE of the fp32 qkv the fp32 form
 * writes; all other outputs identical); ctr_attn_bwd_bf_oproj16 stages them as they are (the same dq / dk / dv as
 * ctr_attn_bwd_bf_oproj on the fp32 qkv) and writes dqkv16 = bf16(dq) | bf16(dk) | bf16(dv) (RNE) -- the dtype of the
 * reference's autocast in-projection output and its grad.  Consumers: ctr_rowgemm_a16, ctr_rowgemm_wgrad_y16.      */
int ctr_attn_layer_fwd_bf16(const float* x, int B, int K, int H, int D, const float* w_in, const float* b_in,
                            const float* rel_w, float* relmean, int tk, float scale, uint32_t drop_key,
                            uint32_t drop_thresh, float drop_scale, uint32_t* mask, const float* w_out, const float* b_out,
                            const float* nw1, float eps, uint16_t* qkv16, float* o, float* mrow, float* lrow, float* h1,
                            float* r1, float* x1, void* stream);
int ctr_attn_bwd_bf_oproj16(const uint16_t* qkv16, const float* o, const float* dh1, const float* w_out, int B, int K,
                            int H, int D, const float* relmean, int tk, float scale, uint32_t drop_key,
                            uint32_t drop_thresh, float drop_scale, const uint32_t* mask, const float* mrow,
                            const float* lrow, uint16_t* dqkv16, float* drel_part, void* stream);
/* amp: bf16 -- the attention half of an encoder layer's backward in one launch, src/models/dare.py:53-62 (out_proj,
 * attention and in_proj backward plus the skip connection): ctr_attn_bwd_bf_oproj16 on one workgroup per sample (all H
 * heads; K <= 64, D = 32, 4 or 8 heads: ctr_attn_bwd_bf_layer_ok) followed, in the same workgroup, by
 * dx = dqkv16 W_in + dh1 with W_in = in_proj_weight (3D x D) -- the bits of ctr_rowgemm_a16(dqkv16, W_in, tb = 0,
 * add = dh1), which it replaces.  dqkv16 is still written (the in-projection's weight grad reads it); drel_part has
 * ONE row per sample (B x (2tk+1)) instead of H / 4.                                                          */
int ctr_attn_bwd_bf_layer_ok(int K, int H, int D);
int ctr_attn_bwd_bf_layer16(const uint16_t* qkv16, const float* o, const float* dh1, const float* w_out,
                            const float* w_in, int B, int K, int H, int D, const float* relmean, int tk, float scale,
                            uint32_t drop_key, uint32_t drop_thresh, float drop_scale, const uint32_t* mask,
                            const float* mrow, const float* lrow, uint16_t* dqkv16, float* drel_part, float* dx,
                            void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fused position-wise FFN + residual + RMSNorm of DAREEncoderLayer, src/models/dare.py:53-70
 * (ffn = Linear(D,FF) -> GELU -> Dropout -> Linear(FF,D); x2 = norm2(x1 + ffn(x1)))       (ffn.hip)
 * The FF-wide activations never reach HBM: the backward recomputes them from x1.
 * ------------------------------------------------------------------------------------------- */
/* flags: CTR_FFN_BF16 (amp: bf16, src/train.py:158-164) -- both products on bf16 MFMA (bf16-rounded operands,
 * fp32 accumulate), GELU / dropout / residual / norms fp32; D in {32, 64}, FF % 32 == 0; the keep-bit
 * mask in the bf16 kernels' own layout (a bf16 forward pairs with a bf16 backward).  wbf: 3*FF*D bf16
 * (6*FF*D bytes) the bf16 forward fills with weight images (W1 | W2^T | W1^T) for the bf16 backward
 * (nullable in an inference-only forward; ignored without the flag)                                    */
#define CTR_FFN_BF16 1
int ctr_ffn_supported(int D, int FF, int flags);   /* fp32: D in {16, 32, 64}, FF % 16 == 0 */
int ctr_ffn_slab_rows(int M, int D, int FF, int flags);   /* workgroups of ctr_ffn_bwd = rows of its grad slab */
int ctr_ffn_mask_words(int M, int FF);         /* uint32 words of the dropout keep-bit mask (16 bits per 16 cols) */
/* y = norm_w * h * r, h = x + (gelu(x W1^T + b1) [dropout] W2^T + b2), r = 1/rms(h).  mask (nullable
 * without dropout) receives the keep bits, chunk-major (FF/16, M) uint16.                           */
int ctr_ffn_fwd(const float* x, int M, int D, int FF, const float* W1, const float* b1, const float* W2,
                const float* b2, const float* norm_w, float eps, uint32_t drop_key, uint32_t drop_thresh,
                float drop_scale, uint32_t* mask, float* y, float* h, float* r, void* wbf, int flags, void* stream);
/* dh = grad wrt h (after ctr_rmsnorm_bwd).  dx = dh + (dact W1); per-workgroup weight-grad slab rows
 * (ld_slab floats): dW1 (FF, D) at 0, db1 (FF) at o_b1, dW2 (D, FF) at o_w2 -- colsum them (the
 * offsets may match the arena layout so one ctr_colsum lands in the grad buffer).  db2 = colsum(dh). */
int ctr_ffn_bwd(const float* x, const float* dh, int M, int D, int FF, const float* W1, const float* b1,
                const float* W2, uint32_t drop_key, uint32_t drop_thresh, float drop_scale, const uint32_t* mask,
                float* dx, float* slab, long ld_slab, int o_b1, int o_w2, const void* wbf, int flags, void* stream);
/* The FFN backward fused with the transformer layer's two RMSNorm backwards (x1 = norm1(h1),
 * h2 = x1 + FFN(x1), x2 = norm2(h2); src/models/dare.py TransformerEncoderLayer norm_first=False):
 * dy = grad wrt x2 -> dh1 = grad wrt h1.  Slab rows (ld_slab floats) hold d norm1.w at o_n1, dW1 at o_w1,
 * db1 at o_b1, dW2 at o_w2, db2 at o_b2, d norm2.w at o_n2 (the arena's parameter order, so one colsum
 * lands all six in the grad buffer).  Replaces ctr_rmsnorm_bwd x2 + ctr_ffn_bwd + the db2 colsum.     */
int ctr_ffn_bwd_norms(const float* x, const float* dy, const float* h2, const float* r2, const float* nw2,
                      const float* h1, const float* r1, const float* nw1, int M, int D, int FF, const float* W1,
                      const float* b1, const float* W2, uint32_t drop_key, uint32_t drop_thresh, float drop_scale,
                      const uint32_t* mask, float* dh1, float* slab, long ld_slab, int o_n1, int o_w1, int o_b1,
                      int o_w2, int o_b2, int o_n2, const void* wbf, int flags, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Row / column ops                                                                (rowops.hip)
 * ------------------------------------------------------------------------------------------- */
/* RMSNorm.forward for long rows (QNN pre_norm, src/models/qnn_alpha.py:110-113) */
int ctr_rmsnorm_fwd(const float* x, long ldx, int M, int N, const float* w, float eps, float* y, long ldy, float* r,
                    void* stream);
/* ... also writing y's bf16 (RNE) image, row stride ldybf (amp: the QNN MLP's [z | inter] GEMM operand); y may be
 * null when every consumer reads the image (the bf16-z pair interaction, ctr_qnn_gram_*_zbf) */
int ctr_rmsnorm_fwd_bf(const float* x, long ldx, int M, int N, const float* w, float eps, float* y, long ldy, float* r,
                       void* ybf, long ldybf, void* stream);
int ctr_rmsnorm_bwd_nparts(int M, int N);
/* RMSNorm backward: dh = w*dy*r - h*r^3/N*sum(w*dy*h) (+ add); dw partials (nparts, N) */
int ctr_rmsnorm_bwd(const float* dy, long ldy, const float* h, long ldh, const float* r, const float* w, int M, int N,
                    float* dh, long lddh, const float* add, long ld_add, float* dw_part, void* stream);
/* LayerNorm (norm options other than "rms": src/models/dare.py:15-18 make_norm -> nn.LayerNorm(d), eps 1e-5) over
 * rows of N <= 16384: y = (x - mean) rstd w + b, mean / rstd saved per row; ybf (nullable) y's bf16 image.
 * Backward: dx = rstd (g w - mean(g w) - xhat mean(g w xhat)) (+ add); dw / db partial rows (nparts, N) each,
 * reduced by ctr_colsum.                                                                          (layernorm.hip) */
int ctr_layernorm_fwd(const float* x, long ldx, int M, int N, const float* w, const float* b, float eps, float* y,
                      long ldy, float* mean, float* rstd, void* ybf, long ldybf, void* stream);
int ctr_layernorm_bwd_nparts(int M, int N);
int ctr_layernorm_bwd(const float* dy, long ldy, const float* x, long ldx, const float* mean, const float* rstd,
                      const float* w, int M, int N, float* dx, long lddx, const float* add, long ld_add,
                      float* dw_part, float* db_part, void* stream);
size_t ctr_colsum_ws_size(int M, int N);
/* out[n] = sum_m X[m,n] / div  (bias grads; div = B gives torch .mean(dim=0)) */
int ctr_colsum(const float* X, long ld, int M, int N, float div, float* out, float* ws, void* stream);
/* several column sums in one launch pair: out_i[n] = sum_m X_i[m,n] / div_i (div 0 or 1: plain sums) for up to
 * CTR_COLSUM_MAXSEG segments (the backward's per-layer weight-grad slabs, summed together once the layers
 * are done).  segs: a HOST array (copied into the launch); every segment needs N and ld multiples of 4 and
 * a 16-byte aligned X (ctr_colsum_multi_ok); ws: ctr_colsum_multi_ws_size bytes.  Deterministic.  */
#define CTR_COLSUM_MAXSEG 16
typedef struct {
  const float* X;
  long ld;
  int M, N;
  float* out;
  float div;
  int pad;
} ctr_colsum_seg_t;
int ctr_colsum_multi_ok(const ctr_colsum_seg_t* seg);
size_t ctr_colsum_multi_ws_size(const ctr_colsum_seg_t* segs, int nseg);
int ctr_colsum_multi(const ctr_colsum_seg_t* segs, int nseg, float* ws, size_t ws_bytes, void* stream);
/* bce_wll_style(logits) + aux_w * bce_wll_style(aux) (src/train.py:71-90,165-168) and d/dlogits, d/daux */
int ctr_loss(const float* z, const float* za, const float* y, int B, float aux_w, float* loss, float* dz, float* dza,
             void* stream);

/* ---------------------------------------------------------------------------------------------
 * QNN-alpha, src/models/qnn_alpha.py                                                  (qnn.hip)
 * ------------------------------------------------------------------------------------------- */
/* U (H,D,R) <-> Ucat (D,H*R) (all heads side by side) */
int ctr_qnn_ucat(const float* src, int H, int D, int R, float* dst, int inverse, void* stream);
/* V (H,R,P) -> block-diagonal Vfull (H*R, H*P) (inverse: extract the diagonal blocks), so the per-head
 * products quad_h @ V_h and their grads are GEMMs                                                    */
int ctr_qnn_vfull(const float* V, int H, int R, int P, float* vfull, int inverse, void* stream);
/* _pair_interaction_all (l.86-97) without forming A = z @ Ucat: per sample b (z rows (F, D)):
 * zsum = sum_f z_f, G = z^T z (D x D), S = zsum @ Ucat, quad = S*S - diag(Ucat^T G Ucat) (QR wide) */
int ctr_qnn_gram_fwd(const float* z, int B, int F, int D, const float* ucat, int QR, float* zsum, float* G,
                     float* S, float* quad, void* stream);
/* backward to z: dz_f = 2 Ucat (dquad o S) - 2 (Ucat diag(dquad) Ucat^T) z_f (+ dz_add, nullable; fp32, or
 * bf16 when add_bf16 -- the MLP's input grad under amp: bf16); DS = dquad o S (for dUcat)           */
int ctr_qnn_gram_bwd(const float* z, int B, int F, int D, const float* ucat, int QR, const float* S,
                     const float* dquad, const void* dz_add, int add_bf16, float* dz, float* DS, void* stream);
/* amp: the pair interaction on bf16(z) (the reference's autocast A = z @ U_h takes z in bf16): z read from the bf16
 * image of [z | inter] (uint16_t = bf16 bits, row stride ldz, 16-byte aligned rows); G = bf16(z)^T bf16(z) on bf16
 * MFMA with fp32 accumulation, zsum the fp32 sum of the bf16 values, S / quad as ctr_qnn_gram_fwd_ex -- the exact
 * sums of the bf16-z function; backward dz_f = 2 w - 2 bf16(M) bf16(z_f) (+ dz_add), M = U diag(dquad) U^T in fp32
 * (dz_add and dz rows: stride ld).  D in {32, 64}; other arguments as the fp32-z forms.                          */
int ctr_qnn_gram_fwd_zbf(const uint16_t* zbf, long ldz, int B, int F, int D, const float* ucat, int QR, float* zsum,
                         float* G, float* S, float* quad, int accumulate, void* stream);
int ctr_qnn_gram_bwd_zbf(const uint16_t* zbf, long ldz, long ld, int B, int F, int D, const float* ucat, int QR,
                         const float* S, const float* dquad, const void* dz_add, int add_bf16, float* dz, float* DS,
                         void* stream);
/* the same over one feature block of the rows (pair_grouping 'block', src/models/qnn_alpha.py:99-116, block slices
 * src/models/wrapper.py:66-75): z (and dz_add, dz) rows of stride ld >= F D, F the block's features; accumulate != 0
 * adds G and quad to what the buffers hold (the blocks' quads summed, qnn_alpha.py:108), zsum / S per block     */
int ctr_qnn_gram_fwd_ex(const float* z, long ld, int B, int F, int D, const float* ucat, int QR, float* zsum, float* G,
                        float* S, float* quad, int accumulate, void* stream);
int ctr_qnn_gram_bwd_ex(const float* z, long ld, int B, int F, int D, const float* ucat, int QR, const float* S,
                        const float* dquad, const void* dz_add, int add_bf16, float* dz, float* DS, void* stream);
/* dst (B, ncols; row stride ld) = add (fp32, or bf16 when add_bf16; row stride ld_add; null: 0) -- the columns of the
 * block form's z rows outside every interaction block                                                  */
int ctr_qnn_passthrough(const void* add, int add_bf16, long ld_add, int B, int ncols, float* dst, long ld, void* stream);
/* dUcat = 2 (T1 - sum_e Ucat[e,c] T[d*D+e, c]) with T1 = zsum^T DS (D x QR), T = G^T dquad (D*D x QR) */
int ctr_qnn_du_combine(const float* T1, const float* T, const float* ucat, int D, int QR, float* ducat,
                       void* stream);
/* SEBlock (l.17-26): gate from the batch mean; scale + QNN dropout (l.120-121) */
int ctr_se_fwd_gate(const float* mean, int C, int Cr, const float* W1, const float* b1, const float* W2,
                    const float* b2, float* g1, float* gate, void* stream);
int ctr_scale_drop(const float* x, int B, int C, const float* gate, uint32_t drop_key, uint32_t drop_thresh,
                   float drop_scale, float* out, long out_ld, void* stream);
int ctr_scale_drop_bf(const float* x, int B, int C, const float* gate, uint32_t drop_key, uint32_t drop_thresh,
                      float drop_scale, float* out, long out_ld, void* obf, long obf_ld, void* stream);
size_t ctr_se_bwd_ws(int B, int C);
/* dout fp32, or bf16 when dout_bf16 (the MLP's input grad under amp: bf16)                          */
int ctr_se_bwd(const void* dout, long dout_ld, int dout_bf16, const float* x, int B, int C, int Cr, const float* gate,
               const float* g1, const float* mean, const float* W1, const float* W2, uint32_t drop_key,
               uint32_t drop_thresh, float drop_scale, float* dx, float* dW1, float* db1, float* dW2, float* db2,
               float* ws, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Embedding-table gradients: deterministic row dedup (rowgrad.hip) -- replaces
 * embedding_dense_backward for src/models/dare.py:89-90 and src/models/wrapper.py:34.
 * keys (n) with 0xFFFFFFFF = dropped; contrib rows at stride ld; outputs sorted unique keys, summed
 * rows (n_uniq x width) and the device count n_uniq.  key_bits: sort bits (max valid key < 2^bits-1).
 * ------------------------------------------------------------------------------------------- */
size_t ctr_rowgrad_ws_size(int n);
int ctr_rowgrad(const uint32_t* keys, const float* contrib, int n, int width, int ld, int key_bits,
                uint32_t* uniq_keys, float* uniq_grad, uint32_t* n_uniq, void* ws, size_t ws_bytes, void* stream);
/* two contribution arrays with the SAME keys (DARE att and rep rows: both keyed by the top-K tokens)
 * share one sort: uniq_a / uniq_b are their per-key sums                                          */
int ctr_rowgrad2(const uint32_t* keys, const float* contrib_a, const float* contrib_b, int n, int width, int ld,
                 int key_bits, uint32_t* uniq_keys, float* uniq_a, float* uniq_b, uint32_t* n_uniq, void* ws,
                 size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fused clip_grad_norm_ + AdamW + EMA over the parameter arena                      (optim.hip)
 * src/train.py:133-139,185-199; torch/optim/adam.py (_single_tensor_adam); src/utils/ema.py:92-131
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  int64_t p_off;            /* element offset of the segment in the arenas (multiple of 4)          */
  int64_t n;                /* elements                                                             */
  int32_t width;            /* row width (kind 1)                                                   */
  int32_t kind;             /* 0 dense grad, 1 sparse table rows, 2 no grad (EMA only)              */
  int64_t g_off;            /* kind 0: offset into the dense grad arena                             */
  const uint32_t* keys;     /* kind 1: sorted unique keys (ctr_rowgrad)                             */
  const float* G;           /* kind 1: summed rows, row stride g_ld                                 */
  const uint32_t* n_uniq;   /* kind 1: device count                                                 */
  int32_t g_ld;
  uint32_t key_base;        /* key of row 0 of this segment                                         */
} ctr_opt_seg_t;
typedef struct {
  int32_t seg, pad;
  int64_t e0, e1;           /* element range [e0, e1) inside the segment (e0 multiple of 4)         */
} ctr_opt_chunk_t;

int ctr_opt_chunk_elems(void);
/* krange: 2*nchunks uint32 scratch (per-chunk key ranges of the sparse segments) */
int ctr_adamw_ema(const ctr_opt_chunk_t* chunks, int nchunks, const ctr_opt_seg_t* segs, uint32_t* krange, float* P,
                  float* M, float* V, float* E, const float* dgrad, const float* coef, float lr, float wd, float beta1,
                  float beta2, float eps, int step, float ema_decay, int do_adam, int do_ema, void* stream);
/* ctr_adamw_ema (do_adam = 1) with hist[tick] = the same tick's scalars recorded in the same launch
 * (ctr_opt_hist_record + ctr_adamw_ema of a lazy FusedAdamW step: one dispatch where those were three; sparse chunks'
 * key ranges are searched inside it, krange is then unused)                                                    */
int ctr_adamw_ema_hist(const ctr_opt_chunk_t* chunks, int nchunks, const ctr_opt_seg_t* segs, uint32_t* krange,
                       float* P, float* M, float* V, float* E, const float* dgrad, const float* coef, float lr, float wd,
                       float beta1, float beta2, float eps, int step, float ema_decay, int do_ema, void* hist, int tick,
                       void* stream);
int ctr_norm_nparts_per_call(void);
int ctr_sqnorm_dense(const float* x, long n, float* part, void* stream);
int ctr_sqnorm_rows(const uint32_t* keys, const float* G, const uint32_t* n_uniq, int width, int ld,
                    uint32_t invalid_key, float* part, void* stream);
/* ctr_sqnorm_dense(x, n) and ctr_sqnorm_rows of each of rows[0 .. nrows) (nrows <= CTR_SQNORM_MAX_ROWS) in one launch:
 * part[0 .. P) the dense partials, part[(1 + j) P ..) table j's, P = ctr_norm_nparts_per_call() -- the same values
 * (bits) the separate calls write, so ctr_clip_finalize over (1 + nrows) P partials gives the same norm.       */
#define CTR_SQNORM_MAX_ROWS 4
typedef struct {
  const uint32_t* keys;
  const float* G;
  const uint32_t* n_uniq;
  int width, ld;
} ctr_sqnorm_rows_t;
int ctr_sqnorm_all(const float* x, long n, const ctr_sqnorm_rows_t* rows, int nrows, uint32_t invalid_key, float* part,
                   void* stream);
/* out[0] = global L2 norm of (summed grads * grad_scale); out[1] = grad_scale * min(1, max_norm/(norm+1e-6))
 * (grad_scale alone if max_norm <= 0) -- the multiplier the AdamW stream applies to raw grads      */
int ctr_clip_finalize(const float* part, int nparts, float max_norm, float grad_scale, float* out, void* stream);
/* data parallel: invalidate slots >= counts[r] of each rank's block of n gathered keys */
int ctr_mask_tail_keys(uint32_t* keys, int n, int world, const uint32_t* counts, void* stream);

/* ---- exact lazy AdamW/EMA for embedding tables (replaces the table part of the dense
 * torch.optim.AdamW.step + ModelEMA.update, src/train.py:195-199, src/utils/ema.py:92-131).
 * Every optimizer tick is recorded in a device history (one 48-byte entry of scalars per tick); each
 * table row remembers the last tick applied to it (last[row]).  A row is brought current -- the
 * skipped ticks replayed with grad 0, bit-identical to the dense stream -- when it is read (forward:
 * ctr_lazy_touch), when it receives a gradient (ctr_lazy_update: replay, then the tick with its grad),
 * or at ctr_lazy_flush (before parameters / moments / EMA are read as a whole).  Untouched rows cost
 * nothing per step, instead of 32 B/element of HBM traffic.                                         */
typedef struct {
  int64_t p_off;     /* arena offset (floats) of the table                                      */
  int64_t rows;      /* rows of the table                                                       */
  int32_t width;     /* row width (floats), 1..64                                               */
  uint32_t key_base; /* first key of this table in its group's compact key space (update only) */
  int32_t* last;     /* per-row last applied tick                                               */
} ctr_lazy_tab_t;

int ctr_opt_hist_entry_bytes(void);
/* hist[tick] = the scalars of one AdamW(+EMA) tick (same arguments as ctr_adamw_ema)              */
int ctr_opt_hist_record(void* hist, int tick, float lr, float wd, float beta1, float beta2, float eps, int step,
                        float ema_decay, int do_adam, int do_ema, void* stream);
/* bring the rows read by a batch up to tick: X (nx, ncols) int32 row ids; per_column == 1: column c
 * indexes tabs[c] (ntabs == ncols); == 2: every entry is a key of the tables' key space (table = last
 * with key_base <= key, row = key - key_base; tabs sorted by key_base); 0: every id is a row of each
 * of the ntabs tables.  E may be NULL (no EMA).                                                     */
int ctr_lazy_touch(const ctr_lazy_tab_t* tabs, int ntabs, const int32_t* X, long nx, int ncols, int per_column,
                   float* P, float* M, float* V, float* E, const void* hist, int tick, void* stream);
/* apply tick to the rows of one compact grad group (sorted unique keys, rows G with leading dim g_ld,
 * *n_uniq valid of at most cap; INVALID keys skipped), replaying each row's skipped ticks first;
 * grads are scaled by *coef (clip multiplier).  tabs sorted by key_base.                           */
int ctr_lazy_update(const ctr_lazy_tab_t* tabs, int ntabs, const uint32_t* keys, const float* G, int g_ld,
                    const uint32_t* n_uniq, long cap, const float* coef, float* P, float* M, float* V, float* E,
                    const void* hist, int tick, void* stream);
/* bring every row of every table up to tick; max_rows = max over tabs of rows                      */
int ctr_lazy_flush(const ctr_lazy_tab_t* tabs, int ntabs, long max_rows, float* P, float* M, float* V, float* E,
                   const void* hist, int tick, void* stream);
/* the DARE table pair {emb_att, emb_rep} (tabs[0], tabs[1], same rows and width): a token's two rows
 * share their last tick, so one wave replays both (att elements in lanes [0, W), rep in [W, 2W)) --
 * no divergence between rows, wave-uniform history loads.  touch: tokens X[0, n); update: unique
 * keys with att grads Ga and rep grads Gb (same keys, as ctr_rowgrad2 produces); flush: all rows.   */
int ctr_lazy_touch_pair(const ctr_lazy_tab_t* tabs, int width, const int32_t* X, long n, float* P, float* M, float* V,
                        float* E, const void* hist, int tick, void* stream);
/* the same with hot_row (>= 0; -1: none): a row most sequences hold (the padding token), claimed once instead of
 * at every position that holds it (widths 4/8/16/32/64; other widths ignore it)                              */
int ctr_lazy_touch_pair_hot(const ctr_lazy_tab_t* tabs, int width, const int32_t* X, long n, int hot_row, float* P,
                            float* M, float* V, float* E, const void* hist, int tick, void* stream);
int ctr_lazy_update_pair(const ctr_lazy_tab_t* tabs, int width, const uint32_t* keys, const float* Ga, const float* Gb,
                         int g_ld, const uint32_t* n_uniq, long cap, const float* coef, float* P, float* M, float* V,
                         float* E, const void* hist, int tick, void* stream);
int ctr_lazy_flush_pair(const ctr_lazy_tab_t* tabs, int width, long rows, float* P, float* M, float* V, float* E,
                        const void* hist, int tick, void* stream);


/* ---- row-sharded embedding tables (BASELINE config 5): row r of a table lives on rank
 * r % world at local row r / world.  Replaces, for tables larger than one GPU, the reference's
 * in-memory nn.Embedding gathers (src/models/dare.py:118-119,138, src/models/wrapper.py:106-112) and
 * embedding_dense_backward with an owner exchange (all-to-alls issued by tossctr/shard.py).
 * Owner-major keys: okey = (id % world) << lbits | local_key; local_key = id / world (sequence) or
 * lbase[c] + id / world (categorical column c).  Valid okeys must be < 2^key_bits - 1.            */
size_t ctr_shard_plan_ws_size(long n);
/* ids X (n = rows*ncols int32; mode 0 sequence tokens, pad_id excluded; mode 1 categorical) -> sorted
 * unique okeys uniq[0, *n_uniq) (INVALID last if a pad was present), remap[i] = 1 + unique index of
 * X[i] (0 for pads), send_counts[w] = unique valid okeys owned by rank w (contiguous runs)          */
int ctr_shard_plan(const int32_t* X, long n, int ncols, int mode, int pad_id, const uint32_t* lbase, int world,
                   int lbits, int key_bits, uint32_t* uniq, uint32_t* n_uniq, int32_t* remap, long long* send_counts,
                   void* ws, size_t ws_bytes, void* stream);
/* owner side: local[i] = okeys[i] & mask                                                            */
int ctr_shard_strip(const uint32_t* okeys, long n, uint32_t mask, int32_t* local, void* stream);
/* owner side: rows of the requested local keys.  mode 0: tabs = {att, rep} (width out_ld), rows to
 * out0 / out1; mode 1: tabs sorted by key_base, row zero-padded to out_ld floats into out0          */
int ctr_shard_gather(const int32_t* local, long n, int mode, const ctr_lazy_tab_t* tabs, int ntabs, const float* P,
                     float* out0, float* out1, int out_ld, void* stream);
/* categorical rows / grads on the wire at their table's width d_c: widths of keys[0, n) (n = *n_ptr when
 * n_ptr is given, INVALID keys width 0; table = last lbase <= key & mask, width dims[table]) ->
 * offsets[0, cap] (exclusive scan; offsets[i+1] - offsets[i] = width of key i) and, with float_counts,
 * the per-owner float sums of owner-major sorted unique keys (the exchange's splits)                 */
size_t ctr_shard_offsets_ws_size(long cap);
int ctr_shard_offsets(const uint32_t* keys, const uint32_t* n_ptr, long n, long cap, uint32_t mask,
                      const uint32_t* lbase, const int32_t* dims, int ntabs, uint32_t* offsets, int world, int lbits,
                      long long* float_counts, void* ws, size_t ws_bytes, void* stream);
/* rows (n, ld) -> packed[offsets[i], offsets[i+1]) ; packed -> rows (n, out_ld) zero-padded           */
int ctr_shard_pack(const float* rows, int ld, long n, const uint32_t* offsets, float* packed, void* stream);
int ctr_shard_unpack(const float* packed, const uint32_t* offsets, long n, float* out, int out_ld, void* stream);
/* one exchange per phase: the per-peer pieces of several arrays (keys of both table groups; att rows, rep
 * rows and packed categorical floats) copied into / out of ONE all-to-all buffer, whose per-peer segments
 * are contiguous.  segs[0, nseg): n 4-byte words from src to dst (host array, passed by value; nseg <= 96
 * per launch, more are issued in chunks)                                                             */
typedef struct {
  const void* src;
  void* dst;
  long long n;
} ctr_seg_t;
int ctr_copy_segments(const ctr_seg_t* segs, int nseg, void* stream);

/* ---- fold-ensemble inference tail (src/infer.py:102-158)                                (infer.hip)
 * p = clip(iso(clip(sigmoid(clip(z/T, +-50))))) with the checkpoint's calibrator (has_T: temperature,
 * n_iso > 0: isotonic thresholds iso_x/iso_y), else clip(sigmoid(z)); clip = [1e-7, 1 - 1e-7]
 * (src/utils/calibration.py:102-110, src/infer.py:108-122)                                        */
int ctr_calibrate(const float* z, int n, float T, int has_T, const float* iso_x, const float* iso_y, int n_iso,
                  float* p, void* stream);
/* ensemble_probs (src/utils/metrics.py:48-86) over P (M models x B): method 0 mean, 1 geom_mean,
 * 2 logit_mean, 3 median, 4 trim_mean (k cut per side), 5 weighted; w (M, nullable) normalised    */
int ctr_ensemble(const float* P, int M, int B, int method, const float* w, int k, float* out, void* stream);

/* misc: prob = sigmoid(logits) (src/models/wrapper.py:175); strided 2-D copy; compact -> dense rows */
int ctr_sigmoid(const float* x, int n, float* y, void* stream);
int ctr_copy2d(const float* src, long lds, float* dst, long ldd, int rows, int cols, void* stream);
/* dst[0, n) = 0 (16-byte aligned dst): the dense grad arena before each backward -- a native kernel where
 * torch's zero_() would put an at::native fill into the step (no reference counterpart: the reference's
 * optimizer.zero_grad(set_to_none=True), src/train.py:157, drops the grads instead)                     */
int ctr_zero_f32(float* dst, long n, void* stream);
/* profiling aid (no reference counterpart): an empty one-wave kernel, step_marker_kernel, launched on the
 * stream so a rocprofv3 kernel trace can be cut at the timed region's boundaries (tools/prof_summary.py) */
int ctr_step_marker(int tag, void* stream);
/* batch assembly from HBM-resident shard columns (replaces ShardedDataset.__getitem__ + collate_sharded,
 * src/data/dataset.py:77-80,98-124): dst[r, :] = src[idx[r], :], rows of row_words 4-byte words     */
int ctr_gather_rows(const void* src, long row_words, const long* idx, int n, void* dst, void* stream);
int ctr_scatter_rows(const uint32_t* keys, const float* G, const uint32_t* n_uniq, int max_uniq, int width, int ld,
                     uint32_t key_base, long n_rows, float* out, void* stream);

/* ---- validation metrics + temperature objective of the K-fold loop (src/utils/metrics.py:5-29,
 * src/utils/calibration.py:23-52)                                                         (metrics.hip)
 * p = sigmoid(z) (f64), or calibrated = 1: clip(sigmoid(clip(f32(z/T), +-50)), 1e-7, 1-1e-7)         */
int ctr_val_prob(const float* z, int n, float T, int calibrated, double* p, void* stream);
size_t ctr_metrics_ws_size(int n);
/* out[0] = sklearn average_precision_score, out[1] = 50:50 weighted logloss, out[2] = #positives (all f64,
 * device); the reference's nan_to_num / clip(1e-12) and one-class rules; deterministic               */
int ctr_ap_wll(const double* p, const float* y, int n, double* out, void* ws, size_t ws_bytes, void* stream);
/* fit_temperature's closure at T: out = {sum y log p, sum (1-y) log(1-p), and their d/dT} over n rows,
 * p = clamp(sigmoid(z/T), 1e-7, 1-1e-7) in f32 (clamped rows: zero grad); ws: ctr_metrics_ws_size */
int ctr_temp_nll(const float* z, const float* y, int n, float T, double* out, void* ws, size_t ws_bytes,
                 void* stream);

/* ---- host-side hot loops of the Parquet -> NPY cache builder (src/data/build_cache_v1.py)  (hostio.cpp)
 * Arrow string columns: offsets (n + 1, int32) into UTF-8 data.  No GPU involved.
 * XXH64(string, seed) per row: the build's stable replacement for polars Series.hash (:104-111,128-129)
 */
int ctr_hash_utf8(const int32_t* offsets, const uint8_t* data, long n, uint64_t seed, uint64_t* out);
/* seq strings -> (n, L) int32 (:149-156): ',' split, empty tokens dropped, int() each, last L tokens
 * right-aligned over pad_id; valid (nullable, 1 byte per row) marks null rows (all pad).  Returns 0, or
 * -(2 + row) for the first row whose token int() would reject / that overflows int32              */
long ctr_parse_seq(const int32_t* offsets, const uint8_t* data, const uint8_t* valid, long n, int L, int pad_id,
                   int32_t* out);

/* seq strings exploded for the co-visitation features (src/features/covis.py:60-80, :174-183): pieces of
 * str.split(",") (empty pieces kept, null seq = no pieces), each a non-strict Int32 cast (null unless
 * [+-]digits within int32), the last top_k kept; an empty list explodes to one null.  _count fills row_ptr
 * (n + 1, int64) and returns the exploded length (or -1); ctr_covis_explode fills tok / pos / ok per
 * element: ok = 1 for a non-null token, pos = (# non-null tokens so far in the row) - 1 (cum_count - 1) */
long ctr_covis_explode_count(const int32_t* offsets, const uint8_t* data, const uint8_t* valid, long n, int top_k,
                             int64_t* row_ptr);
int ctr_covis_explode(const int32_t* offsets, const uint8_t* data, const uint8_t* valid, long n, int top_k,
                      const int64_t* row_ptr, int32_t* tok, int32_t* pos, uint8_t* ok);

/* ---- co-visitation pair statistics and row features (src/features/covis.py:155-292)        (covis.hip)
 * Exploded elements: tok / pos / ok and erow (source row of each element); per source row: tgt (target
 * code, -1 null), tb (time-bin code < 2^tb_bits, -1 null), click (0/1), keep (nullable: all rows).
 * Pair table (device outputs, capacity n): sorted unique keys ((tok ^ 2^31) << 32 | tgt << tb_bits | tb),
 * impr, clicks, w_rec_sum = sum exp(-pos/tau), max_pos, ctr = clip(clip((clicks + p0 S) / (impr + p0 S +
 * (1 - p0) S), 1e-9, 1 - 1e-9), clip_lo, clip_hi), is_lowcount = impr < min_impr; n_pairs and
 * p0 = mean(click) over the kept exploded elements (device scalars).  Deterministic.                  */
size_t ctr_covis_ws_size(long n);
int ctr_covis_pair_stats(const int32_t* tok, const int32_t* pos, const uint8_t* ok, const int32_t* erow, long n,
                         const int32_t* tgt, const int32_t* tb, const uint8_t* click, const uint8_t* keep,
                         int tb_bits, double tau, double prior_strength, double clip_lo, double clip_hi, int min_impr,
                         uint64_t* out_keys, int32_t* out_impr, int64_t* out_clicks, double* out_wsum,
                         int32_t* out_maxpos, double* out_ctr, uint8_t* out_low, int64_t* n_pairs, double* p0,
                         void* ws, size_t ws_bytes, void* stream);
/* per source row in rows[0, nq): its exploded elements (row_ptr) left-joined on the pair table ->
 * out[i*8 + c] = sum_ctr, mean_ctr, max_ctr, top-n mean (polars nulls-first sort, topn <= 16), wmean_ctr
 * = sum(ctr w) / sum(w), sum_impr, max_impr, pnorm_ctr = sqrt(mean ctr^2); nulls -> 0                  */
int ctr_covis_row_features(const int64_t* rows, long nq, const int64_t* row_ptr, const int32_t* tok, const int32_t* pos,
                           const uint8_t* ok, const int32_t* tgt, const int32_t* tb, int tb_bits, double tau,
                           const uint64_t* keys, const double* ctr, const int32_t* impr, const int64_t* n_pairs,
                           int topn, double* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CTR_HIP_H */
