/* C ABI of libstableavatar_hip.so — the MI355X (gfx950) kernels of the StableAvatar hot path
 * (Wan-2.1 1.3B DiT denoise loop + 3-D causal VAE decode).
 *
 * Conventions:
 *  - plain device pointers, element strides, sizes; no framework types cross the ABI;
 *  - every call is asynchronous on the caller's HIP stream (`stream` = hipStream_t, may be NULL);
 *  - the library never allocates; scratch comes from the caller;
 *  - return 0 on success, 1 on a rejected argument, 2000 + hipError_t on a launch failure;
 *    nothing throws across the ABI.  bf16 = IEEE bfloat16 bit pattern (uint16 storage).
 *
 * Each entry point names the reference interface it replaces (paths under the reference repo).
 */
#ifndef STABLEAVATAR_HIP_H
#define STABLEAVATAR_HIP_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Epilogue codes for sa_gemm_bf16 */
enum {
  SA_EPI_BF16 = 0,          /* C(bf16) = A·W^T + bias                                    */
  SA_EPI_GELU_TANH_BF16 = 1,/* C(bf16) = gelu_tanh(A·W^T + bias)   (nn.GELU('tanh'))       */
  SA_EPI_F32 = 2,           /* C(f32)  = A·W^T + bias                                    */
  SA_EPI_RES_F32 = 3,       /* C(f32)  = R + (A·W^T + bias) * gate[row / rows_per_batch] */
  SA_EPI_GELU_ERF_BF16 = 4, /* C(bf16) = gelu_erf(A·W^T + bias)    (nn.GELU())           */
  SA_EPI_SILU_F32 = 5,      /* C(f32)  = silu(A·W^T + bias)                              */
  SA_EPI_BF16_T = 6,        /* C^T(bf16): C[n * ldc + m] = A·W^T + bias (persistent kernel, K % 128 == 0,
                               M % 4 == 0, ldc >= M): the V^T operand of sa_attn_fwd_ex kernel 4 */
  SA_EPI_BF16_TP32 = 7      /* SA_EPI_BF16_T with row 32c + 4q + r at column 32c + 8(q & 3) + 4(q >> 2) + r
                               (ldc >= M rounded up to 32, ldc and strideC % 8 == 0, C 16-B aligned:
                               16-byte stores): the V^T of sa_attn_fwd_ex kernel 3, the
                               DiT's self-attention (wan_fantasy_transformer3d_1B.py:376-379 v projection) */
};

/* nn.Linear on bf16 activations (every Linear of wan/models/wan_fantasy_transformer3d_1B.py
 * :376-379,523-524,550-554,577-578,644-646,832-838,710 and
 * wan/models/vocal_projector_fantasy_1B.py:238-241,313-316,374,393).
 * C[b][M,N] = epi(A[b][M,K] · W[b][N,K]^T).  K % 64 == 0, lda/ldw % 8 == 0, A/W 16-B aligned. */
int sa_gemm_bf16(const void* A, int64_t lda, int64_t strideA, const void* W, int64_t ldw, int64_t strideW,
                 const float* bias, void* C, int64_t ldc, int64_t strideC, int M, int N, int K, int batch,
                 int epilogue, const float* residual, int64_t ldr, int64_t strideR, const float* gate,
                 int64_t gate_bstride, int rows_per_batch, void* stream);

/* sa_gemm_bf16 with the kernel chosen per call (re-entrant A/B; no process-wide state):
 * kernel 0 = auto (the persistent one-wave-per-SIMD kernel where K % 128 == 0 -- 256- or 192-row tiles,
 * whichever takes fewer rounds over the CUs -- else the 8-wave ping-pong), 1 = ping-pong, 2 = persistent
 * 256-row tiles, 3 = persistent 192-row tiles (2 and 3 rejected with 1 when K % 128 != 0);
 * group_m = tile-raster run length (0 = per-kernel default, or env SA_GEMM_GROUP_M read once). */
int sa_gemm_bf16_ex(const void* A, int64_t lda, int64_t strideA, const void* W, int64_t ldw, int64_t strideW,
                    const float* bias, void* C, int64_t ldc, int64_t strideC, int M, int N, int K, int batch,
                    int epilogue, const float* residual, int64_t ldr, int64_t strideR, const float* gate,
                    int64_t gate_bstride, int rows_per_batch, int kernel, int group_m, void* stream);

/* sa_gemm_bf16_ex with A in column panels: A[m, k] = A[(k / a_panel_cols) * a_panel_stride + m * lda +
 * k % a_panel_cols] (a_panel_cols % 64 == 0, batch 1, persistent kernel, EPI_RES_F32).  Reads the
 * sequence-parallel head exchange's receive buffer (one panel per head group) as the O-projection input
 * in place, replacing the all-gather of head outputs into token rows around wan/dist/wan_xfuser.py:72-115
 * (1B:1150-1151 after the USP attention).  a_panel_cols == 0 is sa_gemm_bf16_ex.
 * The buffer must stay readable for sa_gemm_panel_slack_rows() rows (x lda elements) past the last panel's
 * row M - 1: the last panel's tail tile reads those rows (their products are never stored). */
int sa_gemm_bf16_panels(const void* A, int64_t lda, int64_t strideA, const void* W, int64_t ldw, int64_t strideW,
                        const float* bias, void* C, int64_t ldc, int64_t strideC, int M, int N, int K, int batch,
                        int epilogue, const float* residual, int64_t ldr, int64_t strideR, const float* gate,
                        int64_t gate_bstride, int rows_per_batch, int kernel, int group_m, int64_t a_panel_cols,
                        int64_t a_panel_stride, void* stream);

/* The tallest persistent GEMM tile (rows): the slack sa_gemm_bf16_panels needs past its A buffer's last
 * panel row.  No GPU work; wan/dist/wan_xfuser.py has no counterpart (it all-gathers into token rows). */
int sa_gemm_panel_slack_rows(void);

/* attention(q,k,v,...) of wan/models/wan_fantasy_transformer3d_1B.py:158-207 (SDPA path, no mask,
 * q_lens/k_lens ignored) for head_dim 128.  Rows of q/k/v/o are flat [rows, stride] bf16 matrices,
 * head h at column h*head_dim.  segs = device int32 [nseg][4] = {q_row0, q_len, kv_row0, kv_len}:
 * every query row of a segment attends to the kv_len rows starting at kv_row0 (this expresses the
 * batch dimension and the per-frame vocal grouping of :575-586).  accumulate != 0 adds into o. */
int sa_attn_fwd(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg, int max_q_len,
                int heads, int head_dim, int64_t q_stride, int64_t k_stride, int64_t v_stride, int64_t o_stride,
                float scale, int accumulate, void* stream);

/* sa_attn_fwd with the kernel chosen per call (A/B without process-wide state): 0 = auto,
 * 1 = 8 waves x 32 queries on mfma_f32_16x16x32_bf16 (one 256-row workgroup per CU), 2 = the same body
 * with 4 waves x 32 queries (two 128-row workgroups per CU; bit-identical output). */
int sa_attn_fwd_ex(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg,
                   int max_q_len, int heads, int head_dim, int64_t q_stride, int64_t k_stride, int64_t v_stride,
                   int64_t o_stride, float scale, int accumulate, int kernel, void* stream);

/* sa_attn_fwd_ex with an output row map: query row r is written to row o_rows[r] of o (device int32 per
 * query row; NULL = r).  The Ulysses path of usp_attn_forward (wan/dist/wan_xfuser.py:72-115) writes its
 * own token chunk's head outputs straight into the O-projection's input panel and the other chunks into
 * their send slabs. */
int sa_attn_fwd_map(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg,
                    int max_q_len, int heads, int head_dim, int64_t q_stride, int64_t k_stride, int64_t v_stride,
                    int64_t o_stride, float scale, int accumulate, int kernel, const int32_t* o_rows, void* stream);

/* sa_attn_fwd_map on the 8-wave kernel with the keys of the LAST split_tiles (segment, head, 256-query block) tiles
 * split in two halves, each half a workgroup of its own writing fp32 partials (unnormalised O, running max, row sum)
 * to work, and a second launch merging them (log-sum-exp) into o.  For launches whose last round over the CUs is at
 * most half full (the Ulysses N = 8 per-rank shape: 378 tiles on 256 CUs -> the last 122 as 244 halves: 1.5 rounds
 * instead of 2).  work: >= split_tiles * 2 * 256 * (head_dim + 2) floats, 16-B aligned. */
int sa_attn_fwd_split(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg,
                      int max_q_len, int heads, int head_dim, int64_t q_stride, int64_t k_stride, int64_t v_stride,
                      int64_t o_stride, float scale, int accumulate, const int32_t* o_rows, int split_tiles, void* work,
                      int64_t work_bytes, void* stream);

/* The three attentions of WanI2VTalkingCrossAttention.forward (1B:556-603) in one launch: per batch
 * row b, queries q[b*q_len + i] attend to text k/v rows [b*t_len, +t_len), image rows [b*i_len, +i_len)
 * and the vocal rows of their latent frame, [(b*n_frames + f)*nper, +nper) with
 * f = (tok_offset + i) / tokens_per_frame (1B:575-586 on the unsharded sequence); the outputs are
 * summed as bf16((bf16(text) + bf16(img))) + bf16(vocal) (1B:602) into o.  head_dim 128;
 * tokens_per_frame and tok_offset multiples of 256. */
int sa_attn_cross3(const void* q, int64_t q_stride, const void* kt, const void* vt, int64_t t_stride, int t_len,
                   const void* ki, const void* vi, int64_t i_stride, int i_len, const void* kv, const void* vv,
                   int64_t v_stride, int nper, int tokens_per_frame, int n_frames, int tok_offset, void* o,
                   int64_t o_stride, int batch, int q_len, int heads, float scale, void* stream);

/* attention for head dims other than 128 and few queries per segment (vocal projector D=192,
 * vocal_projector_fantasy_1B.py:259-270; 14B :254-267, D = 640; wav2vec2 D = 64): fp32 softmax and math.
 * head_dim <= 256 (multiple of 8): any kv_len (keys in 64-key chunks, online softmax); 256 < head_dim <= 640:
 * exact softmax, kv_len <= 4096. */
int sa_attn_small(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg, int max_q_len,
                  int max_kv_len, int heads, int head_dim, int64_t q_stride, int64_t k_stride, int64_t v_stride,
                  int64_t o_stride, float scale, void* stream);

/* sa_attn_small with the keys of each 32-query chunk split over nsplit workgroups (head_dim <= 256 only), merged by
 * a second launch: for launches with few query chunks (a sequence-parallel rank's vocal projector, 24 workgroups at
 * N = 8).  work: device scratch of nseg * heads * ceil(max_q_len / 32) * nsplit * 32 * (head_dim + 2) floats. */
int sa_attn_small_split(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg,
                        int max_q_len, int max_kv_len, int heads, int head_dim, int64_t q_stride, int64_t k_stride,
                        int64_t v_stride, int64_t o_stride, float scale, int nsplit, void* work, int64_t work_bytes,
                        void* stream);

/* LayerNorm (+affine) (+AdaLN modulate  y*(1+scale[b])+shift[b]) (+gated residual x + y*gate[b]):
 * WanLayerNorm 1B:345-355 and its call sites :675,684,687,721-722; MLPProj LayerNorms :731-734;
 * vocal_projector_fantasy_1B.py:345-347,352,354,386,398.  in/out dtype: 0 = f32, 1 = bf16. */
int sa_layernorm_mod(const void* x, int64_t ldx, int in_dtype, void* out, int64_t ldo, int out_dtype,
                     const float* weight, const float* bias, const float* shift, const float* scale,
                     int64_t mod_bstride, const float* gate, int rows_per_batch, int M, int C, float eps,
                     void* stream);

/* WanRMSNorm over the full width on q (and k) + rope_apply (1B:295-342, :395-396, :403-404) in place.
 * rope = fp32 [1024][head_dim/2][2] (cos, sin) table or NULL (no rotation); token index
 * t = tok_offset + row % rows_per_batch; t >= F*H*W is not rotated (padding, 1B:319). */
int sa_qk_rmsnorm_rope(void* x, int64_t ldx, int q_col, int k_col, const float* wq, const float* wk, int M, int C,
                       int head_dim, float eps, const float* rope, int rows_per_batch, int tok_offset, int F, int H,
                       int W, int n_frame_pairs, int n_height_pairs, void* stream);

/* Sequence-parallel Q/K/V pack (usp_attn_forward's all-to-all input, wan/dist/wan_xfuser.py:72-115): the
 * same RMSNorm + RoPE as sa_qk_rmsnorm_rope on the [M, 3C] QKV rows of this rank's token chunk (q at
 * column 0, k at C, v at 2C), written with v into per-destination slabs instead of in place.  Head group g
 * (C/G columns) of row (CFG row b = b_offset + row / rows_per_batch, token t = row % rows_per_batch) goes
 * as q and as k|v to the slabs of destination my_part*G + g (the exchange sends the k|v slab on to the group's
 * rank of every query part r < R); table = device int64 [G*R][6] {q_ptr, q_ld, q_bstride, kv_ptr, kv_ld,
 * kv_bstride} in elements (v at k + C/G), rows r*G + g with r != my_part unread. */
int sa_qkv_pack(const void* x, int64_t ldx, const float* wq, const float* wk, int M, int C, int head_dim, float eps,
                const float* rope, int rows_per_batch, int tok_offset, int F, int H, int W, int n_frame_pairs,
                int n_height_pairs, const int64_t* table, int G, int R, int my_part, int b_offset, void* stream);

/* cat(x, y, dim=channels) -> Conv3d(k=s=(1,2,2)) im2col (1B:972-976); out = bf16 [B, Lpad, Kpad]. */
int sa_patch_im2col(const void* x, int64_t xb, int64_t xc, int64_t xf, int xcn, const void* y, int64_t yb, int64_t yc,
                    int64_t yf, int ycn, int B, int F, int H, int W, void* out, int Kpad, int Lpad, void* stream);

/* unpatchify (1B:1161-1184): bf16 [B, Lpad, ld_in] -> [B, C, F, H, W] (out_dtype 0 f32 / 1 bf16). */
int sa_unpatchify(const void* in, int64_t ld_in, int Lpad, int B, int C, int F, int H, int W, void* out,
                  int out_dtype, void* stream);

/* sinusoidal_embedding_1d (1B:210-220), fp64 math, fp32 out [B, dim]. */
int sa_timestep_embed(const float* t, int B, int dim, float* out, void* stream);

/* fp32 Linear for <= 8 rows (time MLPs under fp32 autocast, 1B:986-990); act: 0 none, 1 SiLU. */
int sa_small_linear_f32(const float* in, int64_t ldi, int M, const void* W, int64_t ldw, const float* bias,
                        float* out, int64_t ldo, int N, int K, int act_in, int act_out, void* stream);

/* out[l,b,j,c] = mod[l,j,c] + e[b*e_bstride + j*e_jstride + c]   ((self.modulation + e).chunk(6), 1B:672,
 * :721; e_jstride = 0 broadcasts the time embedding over the chunks as Head.forward does) */
int sa_mod_add(const float* mod, const float* e, int64_t e_bstride, int64_t e_jstride, float* out, int L, int B, int J,
               int C, void* stream);

/* CFG combine + FlowMatchEulerDiscreteScheduler.step + overlap blend + scatter of one window
 * (wan/pipeline/wan_inference_long_pipeline.py:751-779). */
int sa_flow_step(const void* latents_all, void* pred_all, const void* noise, int R, int C, int T, int Fw,
                 int64_t HW, int start, float dsigma, float audio_scale, float text_scale, int overlap, int prev_end,
                 const float* weights, int blend, void* stream);

/* out[r] = idx[r] >= 0 ? in[idx[r]] : 0  (split_tensor_with_padding, vocal_projector_fantasy.py:81-131) */
int sa_gather_rows(const void* in, int64_t in_row_bytes, const int32_t* idx, int nrows, void* out,
                   int64_t out_row_bytes, int64_t row_bytes, void* stream);

int sa_fill_f32(float* p, int64_t n, float v, void* stream);
int sa_cast_f32_bf16(const float* in, void* out, int64_t n, void* stream);

/* ---- 3-D causal VAE decoder (wan/models/wan_vae.py), channels-last bf16 activations ---- */

/* CausalConv3d (wan_vae.py:20-39) / Conv2d 3x3 (:80-86) / 1x1 convs over a whole clip as an implicit
 * GEMM: x [T, H/(1+upsample), W/(1+upsample), Cin] -> y [T, H, W, Cout] (+bias) (+residual [T,H,W,Cout]).
 * kt in {1,3} (causal: kt-1 zero frames in front), kh = kw in {1,3} (zero pad (k-1)/2).
 * upsample != 0 reads the input through nearest-exact 2x upsampling (Upsample, :60-66).
 * interleave_half = C > 0 writes time_conv output channel block j of frame t to frame 2t+j
 * (Resample 'upsample3d', :137-140).  w = bf16 [Cout_pad][kt][kh][kw][Cin], Cin % 32 == 0.
 * x_prev (kt > 1, may be null) = the causal cache (CausalConv3d cache_x, :27-36): the kt-1 input
 * frames before frame 0, [kt-1][H'][W'][Cin]; null = zero padding (first chunk / whole clip). */
int sa_conv3d_cl(const void* x, int T, int H, int W, int Cin, int upsample, const void* w, const float* bias, int Cout,
                 int Cout_pad, int kt, int kh, int kw, const void* residual, void* y, int out_f32,
                 int interleave_half, const void* x_prev, void* stream);

/* Encoder downsampling convs on channels-last bf16, fp32 accumulate, bf16 out [T_out][H][W][Cout]:
 * mode 1 = Resample 'downsample2d/3d' spatial part (wan_vae.py:91-100): ZeroPad2d((0,1,0,1)) + 3x3
 *   stride-2 conv per frame, x [T_out][H_in][W_in][Cin] -> H_in/2 x W_in/2, w [Cout_pad][1][3][3][Cin];
 * mode 2 = 'downsample3d' time_conv (3,1,1) stride (2,1,1) without padding (:99, :150-157):
 *   output frame t reads input frames 2t..2t+2 (the caller passes frame 0 separately), w [Cout_pad][3][1][1][Cin]. */
int sa_conv3d_cl_down(const void* x, int T_out, int H_in, int W_in, int Cin, int mode, const void* w,
                      const float* bias, int Cout, int Cout_pad, void* y, void* stream);

/* RMS_norm (wan_vae.py:42-57): x / max(||x||_2, 1e-12) * sqrt(C) * gamma over channels (+SiLU :198-200). */
int sa_vae_rmsnorm_silu(const void* x, void* y, const float* gamma, int64_t rows, int C, int do_silu, void* stream);

/* z [Cz][T*h*w] fp32 -> channels-last bf16 [T*h*w][Cp] of z*std + mean (= z / scale[1] + scale[0], :553-557). */
int sa_vae_input(const float* z, int Cz, int64_t THW, const float* mean, const float* stdv, void* out, int Cp,
                 void* stream);

/* channels-last fp32 [THW][C_stride] -> [C][THW] clamped to [-1,1] (:668); post != 0 also applies
 * decode_latents' /2 + 0.5 and clamp(0,1) (wan_inference_long_pipeline.py:427). */
int sa_vae_output(const float* in, int C_stride, int C, int64_t THW, float* out, int post, void* stream);

/* Encoder output (wan_vae.py:538-545): channels-last fp32 [THW][C_stride] holding mu | log_var ->
 * [2 Cz][THW] fp32 with mu normalised (mu - mean) * (1/std); log_var unchanged. */
int sa_vae_latent_out(const float* in, int C_stride, int Cz, int64_t THW, const float* mean, const float* stdv,
                      float* out, void* stream);

/* row softmax of fp32 scores (scaled) -> bf16 probabilities (AttentionBlock SDPA, wan_vae.py:255-259). */
int sa_softmax_rows(const float* s, int64_t ld_s, void* p, int64_t ld_p, int64_t rows, int n, float scale,
                    void* stream);

/* batched bf16 transpose: out[z][c][r] = in[z][r][c]. */
int sa_transpose_bf16(const void* in, int64_t ld_in, int64_t stride_in, void* out, int64_t ld_out,
                      int64_t stride_out, int rows, int cols, int batch, void* stream);

/* ---- once-per-call encoders: umT5 (wan/models/wan_text_encoder.py) and the
 * CLIP ViT-H/14 visual tower (wan/models/wan_image_encoder.py); their GEMMs are sa_gemm_bf16(_ex) ---- */

/* T5LayerNorm: y(bf16) = bf16(w) * bf16(x * rsqrt(mean(x^2) + eps)); x f32 (in_f32 != 0) or bf16 rows. */
int sa_t5_rmsnorm(const void* x, int64_t ldx, int in_f32, void* y, int64_t ldy, const float* weight, int M, int C,
                  float eps, void* stream);

/* T5Attention softmax: score rows r = (b*heads + h)*rows_per_head + i of s (fp32, unscaled QK^T) get
 * bf16(bf16(s) + bias) with bias = emb[bucket[i][j]][h] (bf16 [num_buckets][heads] relative-position
 * embedding; bucket int32 [rows_per_head][n]; both null = no bias) or finfo(bf16).min where
 * key_mask[b][j] == 0 (int32, null = no mask); fp32 softmax over j < n (<= 2048) -> bf16 p. */
int sa_t5_softmax_bias(const float* s, int64_t ld_s, void* p, int64_t ld_p, int batch, int heads, int rows_per_head,
                       int n, const int32_t* bucket, const void* emb, const int32_t* key_mask, void* stream);

/* T5FeedForward gate: out[m][c] = bf16(fc1 * GELU(gate)) with in = [gate | fc1] bf16 [M][2N] and the
 * reference GELU's per-op bf16 rounding. */
int sa_t5_geglu(const void* in, int64_t ld_in, void* out, int64_t ld_out, int64_t M, int N, void* stream);

/* CLIPModel.forward preprocessing: bicubic (a = -0.75, align_corners False) resize of fp32 planes
 * [C][H][W] in [-1, 1] to [C][S][S], then (x*0.5 + 0.5 - mean[c]) / std[c]. */
int sa_clip_preprocess(const float* in, int C, int H, int W, float* out, int S, const float* mean, const float* stdv,
                       void* stream);

/* Conv2d(C, dim, k = s = P) im2col: fp32 [C][S][S] -> bf16 [1 + (S/P)^2][Kpad], row 0 (class token) zero. */
int sa_clip_patch_im2col(const float* img, int C, int S, int P, void* cols, int Kpad, void* stream);

int sa_cast_bf16_f32(const void* in, float* out, int64_t n, void* stream);

/* ---- wav2vec2 audio encoder: replaces transformers' Wav2Vec2Model called per
 * window at wan_inference_long_pipeline.py:727-729 (loaded at inference.py:475-476).  Transformer layers and
 * the 1-D convs 1-6 run on sa_gemm_bf16 / sa_attn_small; these are the pieces around them. */

/* Feature-encoder conv 0 (Wav2Vec2GroupNormConvLayer: Conv1d(1, C, k, stride, bias=False) -> GroupNorm(C, C)
 * -> GELU) on the fp32 normalised waveform; statistics over all T outputs per channel; bf16 [T][C] out. */
int sa_w2v_conv0_gn_gelu(const float* audio, int n_samples, const float* weight, int C, int k, int stride,
                         const float* gn_weight, const float* gn_bias, float eps, void* out, int T, void* stream);

/* 1-D im2col of a channels-last bf16 [T_in][ldx] tensor for `groups` groups of `cg` channels starting at
 * column col0: out[g][t][j*cg + c] = x[t*stride + j - pad][col0 + g*cg + c] (zero outside the input and for
 * columns >= k*cg up to Kpad).  Wav2Vec2NoLayerNormConvLayer (:conv) and Wav2Vec2PositionalConvEmbedding. */
int sa_conv1d_im2col(const void* x, int64_t ldx, int T_in, int col0, int groups, int cg, int k, int stride, int pad,
                     void* out, int T_out, int Kpad, void* stream);

/* x (f32 [M][ldx]) += y (bf16 [M][ldy]): hidden_states + position_embeddings (Wav2Vec2Encoder.forward). */
int sa_add_f32_bf16(float* x, int64_t ldx, const void* y, int64_t ldy, int M, int N, void* stream);

#ifdef __cplusplus
}
#endif
#endif
