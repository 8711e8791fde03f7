// Kernels of the wav2vec2 audio encoder the pipeline runs once per sliding window (SURVEY.md §8(f) rank 2;
// the reference calls transformers' Wav2Vec2Model(...).last_hidden_state per window at
// wan_inference_long_pipeline.py:727-729, loaded at inference.py:475-476).  The transformer layers and the
// 1-D convolutions 1-6 run as GEMMs on sa_gemm_bf16 (conv = im2col + GEMM with the GELU epilogue), the
// attention on sa_attn_small; these are the pieces around them:
//  * sa_w2v_conv0_gn_gelu : feature-encoder conv 0 (1 input channel, kernel 10, stride 5) in fp32 on the raw
//                           normalised waveform, GroupNorm with one group per channel (statistics over time,
//                           Wav2Vec2GroupNormConvLayer), affine, exact GELU -> bf16 channels-last [T, C]
//  * sa_conv1d_im2col     : channels-last bf16 [T, ld] -> [groups][T_out][Kpad] rows, column j*cg + c holding
//                           input row t*stride + j - pad, channel col0 + g*cg + c (zero outside [0, T_in) and
//                           past k*cg): feature-encoder convs 1-6 and the grouped positional conv
//                           (Wav2Vec2PositionalConvEmbedding, kernel 128, 16 groups, padding 64)
//  * sa_add_f32_bf16      : x(f32) += y(bf16), the positional embedding added to the hidden states
#include "common.h"

namespace {

// one workgroup per output channel: pass 1 the mean over time, pass 2 the variance about it (two-pass, as
// GroupNorm's reference arithmetic), pass 3 normalise + affine + GELU; the 10-tap conv is recomputed in
// every pass (10 MACs per output) instead of keeping the fp32 pre-activation in memory
__global__ __launch_bounds__(256) void w2v_conv0_kernel(const float* audio, const float* w, int k, int stride, int T,
                                                        const float* gw, const float* gb, float eps, bf16* out,
                                                        int C) {
  const int c = blockIdx.x, tid = threadIdx.x;
  __shared__ float red[4];
  __shared__ float wk[64];
  if (tid < k) wk[tid] = w[(long)c * k + tid];
  __syncthreads();
  auto conv = [&](int t) {
    const float* a = audio + (long)t * stride;
    float s = 0.f;
    for (int j = 0; j < k; ++j) s = fmaf(wk[j], a[j], s);
    return s;
  };
  auto block_sum = [&](float v) {
    v = wave_sum(v);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
  };
  float s = 0.f;
  for (int t = tid; t < T; t += 256) s += conv(t);
  const float mean = block_sum(s) / (float)T;
  float q = 0.f;
  for (int t = tid; t < T; t += 256) {
    const float d = conv(t) - mean;
    q = fmaf(d, d, q);
  }
  const float rstd = rsqrtf(block_sum(q) / (float)T + eps);
  const float a = gw[c] * rstd, b = gb[c] - mean * a;
  for (int t = tid; t < T; t += 256) out[(long)t * C + c] = f2bf(gelu_erf(fmaf(conv(t), a, b)));
}

// one thread per 8 consecutive columns of one output row (cg % 8 == 0, Kpad % 8 == 0)
__global__ __launch_bounds__(256) void conv1d_im2col_kernel(const bf16* x, long ldx, int T_in, int col0, int cg,
                                                            int k, int stride, int pad, bf16* out, int T_out,
                                                            int Kpad, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int per_row = Kpad / 8;
  const long r = i / per_row;  // (g * T_out + t)
  const int col = (int)(i % per_row) * 8;
  const int t = (int)(r % T_out), g = (int)(r / T_out);
  bf16x8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = f2bf(0.f);
  if (col < k * cg) {
    const int j = col / cg, c = col % cg;
    const int src = t * stride + j - pad;
    if (src >= 0 && src < T_in) v = *(const bf16x8*)(x + (long)src * ldx + col0 + g * cg + c);
  }
  *(bf16x8*)(out + r * Kpad + col) = v;
}

__global__ __launch_bounds__(256) void add_f32_bf16_kernel(float* x, long ldx, const bf16* y, long ldy, int N,
                                                           long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const long r = i / N;
  const int c = (int)(i % N);
  x[r * ldx + c] += bf2f(y[r * ldy + c]);
}

inline unsigned nblk(long n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

extern "C" int sa_w2v_conv0_gn_gelu(const float* audio, int n_samples, const float* weight, int C, int k, int stride,
                                    const float* gn_weight, const float* gn_bias, float eps, void* out, int T,
                                    void* stream) {
  if (!audio || !weight || !gn_weight || !gn_bias || !out || C <= 0 || k <= 0 || k > 64 || stride <= 0) return SA_ERR_ARG;
  if (T <= 0 || (long)(T - 1) * stride + k > n_samples) return SA_ERR_ARG;
  hipLaunchKernelGGL(w2v_conv0_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, audio, weight, k, stride, T,
                     gn_weight, gn_bias, eps, (bf16*)out, C);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_conv1d_im2col(const void* x, int64_t ldx, int T_in, int col0, int groups, int cg, int k, int stride,
                                int pad, void* out, int T_out, int Kpad, void* stream) {
  if (!x || !out || T_in <= 0 || T_out <= 0 || groups <= 0 || cg <= 0 || k <= 0 || stride <= 0 || pad < 0)
    return SA_ERR_ARG;
  if (cg % 8 || Kpad % 8 || Kpad < k * cg || ldx % 8 || col0 % 8 || col0 + groups * cg > ldx) return SA_ERR_ARG;
  if ((((uintptr_t)x) & 15) || (((uintptr_t)out) & 15)) return SA_ERR_ARG;
  const long total = (long)groups * T_out * (Kpad / 8);
  hipLaunchKernelGGL(conv1d_im2col_kernel, dim3(nblk(total, 256)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x,
                     ldx, T_in, col0, cg, k, stride, pad, (bf16*)out, T_out, Kpad, total);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_add_f32_bf16(float* x, int64_t ldx, const void* y, int64_t ldy, int M, int N, void* stream) {
  if (!x || !y || M <= 0 || N <= 0) return SA_ERR_ARG;
  const long total = (long)M * N;
  hipLaunchKernelGGL(add_f32_bf16_kernel, dim3(nblk(total, 256)), dim3(256), 0, (hipStream_t)stream, x, ldx,
                     (const bf16*)y, ldy, N, total);
  SA_LAUNCH_CHECK();
  return SA_OK;
}
