// Kernels of the once-per-call encoders the pipeline drives: the umT5-XXL text
// encoder (wan/models/wan_text_encoder.py) and the open-CLIP ViT-H/14 visual tower
// (wan/models/wan_image_encoder.py).  Their GEMMs run on sa_gemm_bf16 and the CLIP attention on
// sa_attn_small; these are the row-wise pieces around them, all HBM-bound and tiny next to the DiT:
//  * sa_t5_rmsnorm       : T5LayerNorm (wan_text_encoder.py T5LayerNorm.forward) with its bf16 roundings
//  * sa_t5_softmax_bias  : T5 attention softmax: unscaled scores + relative-position bias (per-head
//                          bucket embedding) + key padding mask, fp32 softmax, bf16 P (T5Attention.forward)
//  * sa_t5_geglu         : T5FeedForward's fc1(x) * GELU_tanh(gate(x)) with the reference's per-op bf16
//                          rounding of its hand-written GELU (GELU.forward)
//  * sa_clip_preprocess  : CLIPModel.forward preprocessing: bicubic resize (F.interpolate, align_corners
//                          False, a = -0.75, clamped taps), *0.5+0.5, Normalize(mean, std)
//  * sa_clip_patch_im2col: Conv2d(3, dim, k=s=patch) as rows of a GEMM, row 0 left zero for the class token
#include "common.h"

namespace {

__device__ __forceinline__ float rbf(float x) { return bf2f(f2bf(x)); }

template <int IN_F32>
__global__ __launch_bounds__(256) void t5_rmsnorm_kernel(const void* x, long ldx, bf16* y, long ldy, const float* w,
                                                         int C, float eps) {
  const long row = blockIdx.x;
  const int tid = threadIdx.x;
  __shared__ float red[4];
  float ss = 0.f;
  for (int c = tid; c < C; c += 256) {
    const float v = IN_F32 ? ((const float*)x)[row * ldx + c] : bf2f(((const bf16*)x)[row * ldx + c]);
    ss += v * v;
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float r = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)C + eps);
  for (int c = tid; c < C; c += 256) {
    const float v = IN_F32 ? ((const float*)x)[row * ldx + c] : bf2f(((const bf16*)x)[row * ldx + c]);
    // x * rsqrt(mean(x^2) + eps) in fp32, cast to the bf16 weight dtype, then weight * x in bf16
    y[row * ldy + c] = f2bf(rbf(w[c]) * rbf(v * r));
  }
}

// one workgroup per score row r = (b * heads + h) * rows_per_head + i
__global__ __launch_bounds__(256) void t5_softmax_bias_kernel(const float* s, long lds_, bf16* p, long ldp, int n,
                                                              int rows_per_head, int heads, const int* bucket,
                                                              const bf16* emb, const int* key_mask) {
  const long row = blockIdx.x;
  const int i = (int)(row % rows_per_head);
  const int h = (int)((row / rows_per_head) % heads);
  const int b = (int)(row / ((long)rows_per_head * heads));
  const float* sr = s + row * lds_;
  __shared__ float red[4];
  __shared__ float v[2048];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float neg = -3.3895313892515355e38f;  // torch.finfo(torch.bfloat16).min
  float mx = -INFINITY;
  for (int j = tid; j < n; j += 256) {
    // einsum output (bf16) + attn_bias (bf16: relative-position bias, or finfo.min where the key is masked)
    float bias = 0.f;
    if (key_mask && key_mask[(long)b * n + j] == 0)
      bias = neg;
    else if (bucket)
      bias = bf2f(emb[(long)bucket[(long)i * n + j] * heads + h]);
    const float t = rbf(rbf(sr[j]) + bias);
    v[j] = t;
    mx = fmaxf(mx, t);
  }
  mx = wave_max(mx);
  if (lane == 0) red[wv] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int j = tid; j < n; j += 256) {
    const float e = __expf(v[j] - mx);
    v[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  if (lane == 0) red[wv] = sum;
  __syncthreads();
  const float inv = 1.f / (red[0] + red[1] + red[2] + red[3]);
  for (int j = tid; j < n; j += 256) p[row * ldp + j] = f2bf(v[j] * inv);
}

// GELU.forward of wan_text_encoder.py on a bf16 tensor: every torch op rounds to bf16
//   0.5 * x * (1.0 + tanh(sqrt(2/pi) * (x + 0.044715 * x^3)))
__device__ __forceinline__ float t5_gelu_bf16(float x) {
  const float half_x = rbf(0.5f * x);
  const float x3 = rbf(x * x * x);
  const float inner = rbf(x + rbf(0.044715f * x3));
  const float th = rbf(tanhf(rbf(0.7978845608028654f * inner)));
  return rbf(half_x * rbf(1.0f + th));
}

__global__ __launch_bounds__(256) void t5_geglu_kernel(const bf16* in, long ldi, bf16* out, long ldo, long M, int N) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= M * N) return;
  const long r = idx / N;
  const int c = (int)(idx % N);
  const float g = t5_gelu_bf16(bf2f(in[r * ldi + c]));
  const float f = bf2f(in[r * ldi + N + c]);
  out[r * ldo + c] = f2bf(f * g);
}

__device__ __forceinline__ float cubic_w(float t, int k) {
  // PyTorch upsample_bicubic2d cubic convolution coefficients, A = -0.75
  const float A = -0.75f;
  auto c1 = [&](float x) { return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f; };
  auto c2 = [&](float x) { return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A; };
  switch (k) {
    case 0: return c2(t + 1.f);
    case 1: return c1(t);
    case 2: return c1(1.f - t);
    default: return c2(2.f - t);
  }
}

// in: fp32 planes [C][Hin][Win] (the reference frame in [-1, 1]); out fp32 [C][S][S]
__global__ __launch_bounds__(256) void clip_preprocess_kernel(const float* in, int C, int Hin, int Win, float* out, int S,
                                                              const float* mean, const float* stdv) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)C * S * S) return;
  const int c = (int)(idx / ((long)S * S));
  const int oy = (int)((idx / S) % S), ox = (int)(idx % S);
  const float sy = (float)Hin / S, sx = (float)Win / S;
  const float fy = (oy + 0.5f) * sy - 0.5f, fx = (ox + 0.5f) * sx - 0.5f;
  const int iy = (int)floorf(fy), ix = (int)floorf(fx);
  const float ty = fy - iy, tx = fx - ix;
  const float* pl = in + (long)c * Hin * Win;
  float acc = 0.f;
#pragma unroll
  for (int ky = 0; ky < 4; ++ky) {
    const int yy = min(max(iy - 1 + ky, 0), Hin - 1);
    float rowv = 0.f;
#pragma unroll
    for (int kx = 0; kx < 4; ++kx) {
      const int xx = min(max(ix - 1 + kx, 0), Win - 1);
      rowv += pl[(long)yy * Win + xx] * cubic_w(tx, kx);
    }
    acc += rowv * cubic_w(ty, ky);
  }
  out[idx] = ((acc * 0.5f + 0.5f) - mean[c]) / stdv[c];
}

// img fp32 [C][S][S] -> bf16 cols [1 + (S/P)^2][Kpad]; row 0 (class token) and columns >= C*P*P zero;
// column order (c, ky, kx) = the Conv2d weight [dim][C][P][P] flattened
__global__ __launch_bounds__(256) void clip_patch_im2col_kernel(const float* img, int C, int S, int P, bf16* cols,
                                                                int Kpad) {
  const int g = S / P;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)(1 + g * g) * Kpad;
  if (idx >= total) return;
  const int row = (int)(idx / Kpad), k = (int)(idx % Kpad);
  float v = 0.f;
  if (row > 0 && k < C * P * P) {
    const int pidx = row - 1, py = pidx / g, px = pidx % g;
    const int c = k / (P * P), ky = (k / P) % P, kx = k % P;
    v = img[((long)c * S + py * P + ky) * S + px * P + kx];
  }
  cols[idx] = f2bf(v);
}

__global__ __launch_bounds__(256) void cast_bf16_f32_kernel(const bf16* in, float* out, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = bf2f(in[i]);
}

inline unsigned nblk(long n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

extern "C" int sa_t5_rmsnorm(const void* x, int64_t ldx, int in_f32, void* y, int64_t ldy, const float* weight, int M,
                             int C, float eps, void* stream) {
  if (!x || !y || !weight || M <= 0 || C <= 0) return SA_ERR_ARG;
  if (in_f32)
    hipLaunchKernelGGL(t5_rmsnorm_kernel<1>, dim3(M), dim3(256), 0, (hipStream_t)stream, x, ldx, (bf16*)y, ldy, weight,
                       C, eps);
  else
    hipLaunchKernelGGL(t5_rmsnorm_kernel<0>, dim3(M), dim3(256), 0, (hipStream_t)stream, x, ldx, (bf16*)y, ldy, weight,
                       C, eps);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_t5_softmax_bias(const float* s, int64_t ld_s, void* p, int64_t ld_p, int batch, int heads,
                                  int rows_per_head, int n, const int32_t* bucket, const void* emb,
                                  const int32_t* key_mask, void* stream) {
  if (!s || !p || batch <= 0 || heads <= 0 || rows_per_head <= 0 || n <= 0 || n > 2048) return SA_ERR_ARG;
  if ((bucket == nullptr) != (emb == nullptr)) return SA_ERR_ARG;
  const long rows = (long)batch * heads * rows_per_head;
  hipLaunchKernelGGL(t5_softmax_bias_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, s, ld_s,
                     (bf16*)p, ld_p, n, rows_per_head, heads, bucket, (const bf16*)emb, key_mask);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_t5_geglu(const void* in, int64_t ld_in, void* out, int64_t ld_out, int64_t M, int N, void* stream) {
  if (!in || !out || M <= 0 || N <= 0) return SA_ERR_ARG;
  hipLaunchKernelGGL(t5_geglu_kernel, dim3(nblk(M * N, 256)), dim3(256), 0, (hipStream_t)stream, (const bf16*)in,
                     ld_in, (bf16*)out, ld_out, M, N);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_clip_preprocess(const float* in, int C, int H, int W, float* out, int S, const float* mean,
                                  const float* stdv, void* stream) {
  if (!in || !out || !mean || !stdv || C <= 0 || H <= 0 || W <= 0 || S <= 0) return SA_ERR_ARG;
  hipLaunchKernelGGL(clip_preprocess_kernel, dim3(nblk((long)C * S * S, 256)), dim3(256), 0, (hipStream_t)stream, in,
                     C, H, W, out, S, mean, stdv);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_clip_patch_im2col(const float* img, int C, int S, int P, void* cols, int Kpad, void* stream) {
  if (!img || !cols || C <= 0 || P <= 0 || S % P || Kpad < C * P * P) return SA_ERR_ARG;
  const int g = S / P;
  hipLaunchKernelGGL(clip_patch_im2col_kernel, dim3(nblk((long)(1 + g * g) * Kpad, 256)), dim3(256), 0,
                     (hipStream_t)stream, img, C, S, P, (bf16*)cols, Kpad);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_cast_bf16_f32(const void* in, float* out, int64_t n, void* stream) {
  if (!in || !out || n <= 0) return SA_ERR_ARG;
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, (const bf16*)in, out,
                     n);
  SA_LAUNCH_CHECK();
  return SA_OK;
}
