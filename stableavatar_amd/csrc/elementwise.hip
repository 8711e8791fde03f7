// Small / memory-bound kernels around the DiT GEMMs and the sampler step.
//  sa_patch_im2col     : cat(x, y) + Conv3d(k=s=(1,2,2)) as an im2col feeding the GEMM   (1B:972-983)
//  sa_unpatchify       : Head output [B,L,64] -> [B,16,F,2h,2w]  einsum fhwpqrc->cfphqwr   (1B:1161-1184)
//  sa_timestep_embed   : sinusoidal_embedding_1d in fp64                                 (1B:210-220)
//  sa_small_linear_f32 : fp32 Linear for the M<=8-row time MLPs (fp32 autocast)          (1B:986-990)
//  sa_mod_add          : per-layer AdaLN vectors  e = modulation + e0                    (1B:672,721)
//  sa_flow_step        : CFG combine + FlowMatch Euler step + overlap blend + scatter    (pipeline:751-779)
//  sa_gather_rows      : row gather with zero rows (vocal frame split)                   (vocal_projector_fantasy.py:81-131)
//  sa_fill_f32, sa_cast_f32_bf16
#include "common.h"

namespace {

__global__ void patch_im2col_kernel(const bf16* x, long xb, long xc, long xf, int xcn, const bf16* y, long yb, long yc,
                                    long yf, int ycn, int B, int F, int H, int W, bf16* out, int Kpad, int Lpad) {
  const int hp = H / 2, wp = W / 2;
  const long ntok = (long)B * Lpad;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;  // one thread per (token, 8-col chunk)
  const int nchunk = Kpad / 8;
  if (idx >= ntok * nchunk) return;
  const long tok = idx / nchunk;
  const int ch = idx % nchunk;
  const int b = tok / Lpad, t = tok % Lpad;
  bf16x8 o;
  const int real = F * hp * wp;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = ch * 8 + j;
    float v = 0.f;
    const int c = k >> 2, kh = (k >> 1) & 1, kw = k & 1;
    if (t < real && c < xcn + ycn) {
      const int f = t / (hp * wp), hh = (t / wp) % hp, ww = t % wp;
      const long sp = (long)(2 * hh + kh) * W + (2 * ww + kw);
      if (c < xcn) v = bf2f(x[b * xb + c * xc + f * xf + sp]);
      else v = bf2f(y[b * yb + (c - xcn) * yc + f * yf + sp]);
    }
    o[j] = f2bf(v);
  }
  *(bf16x8*)(out + tok * Kpad + ch * 8) = o;
}

template <typename TO>
__global__ void unpatchify_kernel(const bf16* in, long ld_in, int Lpad, int B, int C, int F, int H, int W, TO* out) {
  // out [B, C, F, H, W] with H, W the latent (un-patched) sizes
  const long n = (long)B * C * F * H * W;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n) return;
  const int w = idx % W, h = (idx / W) % H, f = (idx / ((long)W * H)) % F;
  const int c = (idx / ((long)W * H * F)) % C, b = idx / ((long)W * H * F * C);
  const int hp = H / 2, wp = W / 2;
  const long tok = (long)f * hp * wp + (h >> 1) * wp + (w >> 1);
  const int col = ((h & 1) * 2 + (w & 1)) * C + c;
  out[idx] = (TO)bf2f(in[((long)b * Lpad + tok) * ld_in + col]);
}

__global__ void timestep_embed_kernel(const float* t, int B, int dim, float* out) {
  const int b = blockIdx.x, i = threadIdx.x;
  const int half = dim / 2;
  if (i >= half) return;
  const double pos = (double)t[b];
  const double fr = pow(10000.0, -(double)i / (double)half);
  const double s = pos * fr;
  out[b * dim + i] = (float)cos(s);
  out[b * dim + half + i] = (float)sin(s);
}

// out[m, n] = act_out( act_in(in[m,:]) . W[n,:] + bias[n] ), one wave per output column n
__global__ __launch_bounds__(256) void small_linear_kernel(const float* in, long ldi, int M, const bf16* W, long ldw,
                                                           const float* bias, float* out, long ldo, int N, int K,
                                                           int act_in, int act_out) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (n >= N) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bf16* w = W + (long)n * ldw;
  for (int k = lane * 8; k < K; k += 512) {
    bf16x8 wv = *(const bf16x8*)(w + k);
#pragma unroll
    for (int m = 0; m < 8; ++m)
      if (m < M) {
        const float* ip = in + (long)m * ldi + k;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float xv = ip[j];
          if (act_in == 1) xv = silu(xv);
          acc[m] = fmaf(xv, bf2f(wv[j]), acc[m]);
        }
      }
  }
#pragma unroll
  for (int m = 0; m < 8; ++m)
    if (m < M) {
      float v = wave_sum(acc[m]);
      if (lane == 0) {
        v += bias ? bias[n] : 0.f;
        if (act_out == 1) v = silu(v);
        out[(long)m * ldo + n] = v;
      }
    }
}

// out[l, b, j, c] = mod[l, j, c] + e[b, j, c]      (e broadcast over layers, mod over batch)
__global__ void mod_add_kernel(const float* mod, const float* e, long eb, long ej, float* out, int L, int B, int J,
                               int C) {
  const long n = (long)L * B * J * C;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n) return;
  const int c = idx % C, j = (idx / C) % J, b = (idx / ((long)C * J)) % B, l = idx / ((long)C * J * B);
  out[idx] = mod[((long)l * J + j) * C + c] + e[b * eb + j * ej + c];
}

// One sampler step for one window (pipeline:751-779):
//   v   = u + a*(d-u) + t*(c-d)                      (bf16 noise_pred rows u/d/c)   if cfg
//   x1  = bf16( x0 + bf16((sigma_next - sigma) * v) )  (FlowMatchEuler step, sample upcast to fp32)
//   x1[j] = bf16( x1[j]*w_j + prev[j]*(1-w_j) )      for the first `overlap` frames when blending
//   dst[frame_start + j] = x1[j]
// Layout: latents [C, T, HW] (batch 1); noise_pred [R, C, Fw, HW]; window = frames [s, s+Fw).
__global__ void flow_step_kernel(const bf16* latents_all, bf16* pred_all, const bf16* noise, int R, int C, int T,
                                 int Fw, long HW, int start, float dsigma, float audio_scale, float text_scale,
                                 int overlap, int prev_end, const float* wts, int blend) {
  const long n = (long)C * Fw * HW;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n) return;
  const long p = idx % HW;
  const int f = (idx / HW) % Fw, c = idx / (HW * Fw);
  const long nidx = ((long)c * Fw + f) * HW + p;
  float v;
  if (R == 3) {
    // reference math is bf16 elementwise; round each partial like torch does on bf16 tensors
    const float u = bf2f(noise[nidx]);
    const float d = bf2f(noise[(long)C * Fw * HW + nidx]);
    const float cc = bf2f(noise[2L * C * Fw * HW + nidx]);
    const float t1 = bf2f(f2bf(bf2f(f2bf(d - u)) * audio_scale));
    const float t2 = bf2f(f2bf(bf2f(f2bf(cc - d)) * text_scale));
    v = bf2f(f2bf(bf2f(f2bf(u + t1)) + t2));
  } else {
    v = bf2f(noise[nidx]);
  }
  const int fa = (start + f) % T;
  const float x0 = bf2f(latents_all[((long)c * T + fa) * HW + p]);
  float x1 = bf2f(f2bf(x0 + bf2f(f2bf(dsigma * v))));  // 0-d fp32 * bf16 tensor -> bf16, then + fp32 sample
  if (blend && f < overlap) {
    const float w = bf2f(f2bf(wts[f]));
    const int fp = (prev_end - overlap + f) % T;
    const float pv = bf2f(pred_all[((long)c * T + fp) * HW + p]);
    const float a1 = bf2f(f2bf(x1 * w));
    const float a2 = bf2f(f2bf(pv * bf2f(f2bf(1.f - w))));
    x1 = bf2f(f2bf(a1 + a2));
  }
  pred_all[((long)c * T + fa) * HW + p] = f2bf(x1);
}

__global__ void gather_rows_kernel(const char* in, long in_row_bytes, const int* idx, int nrows, char* out,
                                   long out_row_bytes, long row_bytes) {
  const int r = blockIdx.x;
  if (r >= nrows) return;
  const int src = idx[r];
  for (long i = threadIdx.x * 4; i < row_bytes; i += blockDim.x * 4) {
    unsigned v = 0;
    if (src >= 0) v = *(const unsigned*)(in + (long)src * in_row_bytes + i);
    *(unsigned*)(out + (long)r * out_row_bytes + i) = v;
  }
}

__global__ void fill_f32_kernel(float* p, long n, float v) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < n) p[idx] = v;
}
__global__ void cast_f32_bf16_kernel(const float* in, bf16* out, long n) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < n) out[idx] = f2bf(in[idx]);
}

inline unsigned nblk(long n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace

extern "C" int sa_patch_im2col(const void* x, int64_t xb, int64_t xc, int64_t xf, int xcn, const void* y, int64_t yb,
                               int64_t yc, int64_t yf, int ycn, int B, int F, int H, int W, void* out, int Kpad,
                               int Lpad, void* stream) {
  if (!x || !out || Kpad % 8 || Kpad < 4 * (xcn + ycn) || H % 2 || W % 2) return SA_ERR_ARG;
  if (ycn > 0 && !y) return SA_ERR_ARG;
  if ((long)F * (H / 2) * (W / 2) > Lpad) return SA_ERR_ARG;
  const long n = (long)B * Lpad * (Kpad / 8);
  hipLaunchKernelGGL(patch_im2col_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, xb,
                     xc, xf, xcn, (const bf16*)y, yb, yc, yf, ycn, B, F, H, W, (bf16*)out, Kpad, Lpad);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_unpatchify(const void* in, int64_t ld_in, int Lpad, int B, int C, int F, int H, int W, void* out,
                             int out_dtype, void* stream) {
  if (!in || !out || H % 2 || W % 2) return SA_ERR_ARG;
  const long n = (long)B * C * F * H * W;
  if (out_dtype == 1)
    hipLaunchKernelGGL(unpatchify_kernel<bf16>, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)in, ld_in, Lpad, B, C, F, H, W, (bf16*)out);
  else
    hipLaunchKernelGGL(unpatchify_kernel<float>, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)in, ld_in, Lpad, B, C, F, H, W, (float*)out);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_timestep_embed(const float* t, int B, int dim, float* out, void* stream) {
  if (!t || !out || dim % 2 || dim > 2048) return SA_ERR_ARG;
  hipLaunchKernelGGL(timestep_embed_kernel, dim3(B), dim3(dim / 2), 0, (hipStream_t)stream, t, B, dim, out);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_small_linear_f32(const float* in, int64_t ldi, int M, const void* W, int64_t ldw, const float* bias,
                                   float* out, int64_t ldo, int N, int K, int act_in, int act_out, void* stream) {
  if (!in || !W || !out || M <= 0 || M > 8 || K % 8 || ldw % 8) return SA_ERR_ARG;
  hipLaunchKernelGGL(small_linear_kernel, dim3(nblk(N, 4)), dim3(256), 0, (hipStream_t)stream, in, ldi, M,
                     (const bf16*)W, ldw, bias, out, ldo, N, K, act_in, act_out);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_mod_add(const float* mod, const float* e, int64_t e_bstride, int64_t e_jstride, float* out, int L,
                          int B, int J, int C, void* stream) {
  if (!mod || !e || !out) return SA_ERR_ARG;
  const long n = (long)L * B * J * C;
  hipLaunchKernelGGL(mod_add_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, mod, e, e_bstride, e_jstride,
                     out, L, B, J, C);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_flow_step(const void* latents_all, void* pred_all, const void* noise, int R, int C, int T, int Fw,
                            int64_t HW, int start, float dsigma, float audio_scale, float text_scale, int overlap,
                            int prev_end, const float* weights, int blend, void* stream) {
  if (!latents_all || !pred_all || !noise || (R != 1 && R != 3) || Fw > T) return SA_ERR_ARG;
  if (blend && (!weights || overlap <= 0 || overlap > Fw)) return SA_ERR_ARG;
  const long n = (long)C * Fw * HW;
  hipLaunchKernelGGL(flow_step_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)latents_all, (bf16*)pred_all, (const bf16*)noise, R, C, T, Fw, HW, start, dsigma,
                     audio_scale, text_scale, overlap, prev_end, weights, blend);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_gather_rows(const void* in, int64_t in_row_bytes, const int32_t* idx, int nrows, void* out,
                              int64_t out_row_bytes, int64_t row_bytes, void* stream) {
  if (!in || !out || !idx || row_bytes % 4 || in_row_bytes % 4 || out_row_bytes % 4) return SA_ERR_ARG;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(nrows), dim3(256), 0, (hipStream_t)stream, (const char*)in,
                     in_row_bytes, idx, nrows, (char*)out, out_row_bytes, row_bytes);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_fill_f32(float* p, int64_t n, float v, void* stream) {
  if (!p || n < 0) return SA_ERR_ARG;
  if (n == 0) return SA_OK;
  hipLaunchKernelGGL(fill_f32_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, p, n, v);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_cast_f32_bf16(const float* in, void* out, int64_t n, void* stream) {
  if (!in || !out || n < 0) return SA_ERR_ARG;
  if (n == 0) return SA_OK;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, in, (bf16*)out, n);
  SA_LAUNCH_CHECK();
  return SA_OK;
}
