// bf16 "NT" GEMM for every nn.Linear on the StableAvatar DiT / VAE path:
//   C[M,N] = A[M,K] · W[N,K]^T  (+bias, fused epilogue)
// W is the PyTorch Linear weight [out,in] as stored in the checkpoint, so both operands
// are K-contiguous and every MFMA fragment is one 16-byte LDS read.
// Tile 256x256x64, 8 waves (2M x 4N), mfma_f32_16x16x32_bf16, global_load_lds (16B/lane)
// staging into a 2-deep LDS ring with an XOR swizzle, XCD-aware block order.
// Replaces the aten::addmm sites listed in SURVEY.md §2.2 (wan_fantasy_transformer3d_1B.py
// :376-379,550-554,577-578,644-646,832-838,710, vocal_projector_fantasy_1B.py:238-241,313-316).
#include "common.h"

namespace {

enum { EPI_BF16 = 0, EPI_GELU_BF16 = 1, EPI_F32 = 2, EPI_RES_F32 = 3, EPI_GELU_ERF_BF16 = 4, EPI_SILU_F32 = 5 };

struct GemmArgs {
  const bf16* A; long lda; long sA;
  const bf16* W; long ldw; long sW;
  const float* bias;
  void* C; long ldc; long sC;
  const float* R; long ldr; long sR;     // residual (EPI_RES_F32); may alias C
  const float* gate; long gate_bstride;  // gate[(m / rows_per_batch) * gate_bstride + n]
  int rows_per_batch;
  int M, N, K;
};

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int STAGE_BYTES = (BM + BN) * BK * 2;  // 64 KB
constexpr int LDS_BYTES = 2 * STAGE_BYTES;       // 128 KB

// byte offset of 16-byte chunk c of row r in a [rows][64] bf16 tile (128-B rows)
__device__ __forceinline__ int swz128(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int EPI>
__global__ __launch_bounds__(512) void gemm_nt_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nm = (g.M + BM - 1) / BM, nn = (g.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, nm * nn);
  const int mt = wg / nn, nt = wg % nn;
  const int m0 = mt * BM, n0 = nt * BN;
  const long bz = blockIdx.z;
  const bf16* A = g.A + bz * g.sA;
  const bf16* W = g.W + bz * g.sW;

  // per-lane global element offsets of this lane's 4 A and 4 W staging chunks (k0 added per tile)
  long aoff[4], woff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wave * 4 + i) * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);  // source-side swizzle, LDS image stays lane-linear
    const int ar = min(m0 + row, g.M - 1), wr = min(n0 + row, g.N - 1);
    aoff[i] = (long)ar * g.lda + chunk * 8;
    woff[i] = (long)wr * g.ldw + chunk * 8;
  }
  auto stage = [&](int kt, int buf) {
    char* base = smem + buf * STAGE_BYTES;
    const long k0 = (long)kt * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_global_load_lds((const void*)(A + aoff[i] + k0), LDS_PTR(base + (wave * 4 + i) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(W + woff[i] + k0), LDS_PTR(base + BM * BK * 2 + (wave * 4 + i) * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BK;
  stage(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1);
    const char* As = smem + (kt & 1) * STAGE_BYTES;
    const char* Bs = As + BM * BK * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 a[8], b[4];
      const int c = kk * 4 + (lane >> 4);
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int row = wm * 128 + m * 16 + (lane & 15);
        a[m] = *(const bf16x8*)(As + swz128(row, c));
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int row = wn * 64 + n * 16 + (lane & 15);
        b[n] = *(const bf16x8*)(Bs + swz128(row, c));
      }
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], b[n], acc[m][n], 0, 0, 0);
    }
  }
  __syncthreads();

  // epilogue: per wave, stage one 16x64 fp32 strip at a time through LDS, then 16 contiguous
  // columns per lane -> vector stores
  float* strip = (float*)(smem + wave * (16 * 68 * 4));
  const int er = lane >> 2, ec = (lane & 3) * 16;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) strip[((lane >> 4) * 4 + i) * 68 + n * 16 + (lane & 15)] = acc[m][n][i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    float v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 t = *(const f32x4*)(strip + er * 68 + ec + j * 4);
      v[j * 4 + 0] = t[0]; v[j * 4 + 1] = t[1]; v[j * 4 + 2] = t[2]; v[j * 4 + 3] = t[3];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const int grow = m0 + wm * 128 + m * 16 + er;
    const int gcol = n0 + wn * 64 + ec;
    if (grow >= g.M) continue;
    const bool full = (gcol + 16 <= g.N);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int cc = gcol + j;
      float b = (g.bias && cc < g.N) ? g.bias[cc] : 0.f;
      v[j] += b;
      if (EPI == EPI_GELU_BF16) v[j] = gelu_tanh(v[j]);
      if (EPI == EPI_GELU_ERF_BF16) v[j] = gelu_erf(v[j]);
      if (EPI == EPI_SILU_F32) v[j] = silu(v[j]);
    }
    if (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_GELU_ERF_BF16) {
      bf16* C = (bf16*)g.C + bz * g.sC + (long)grow * g.ldc + gcol;
      if (full) {
        bf16x8 o0, o1;
#pragma unroll
        for (int j = 0; j < 8; ++j) { o0[j] = f2bf(v[j]); o1[j] = f2bf(v[8 + j]); }
        *(bf16x8*)C = o0;
        *(bf16x8*)(C + 8) = o1;
      } else {
        for (int j = 0; j < 16; ++j) if (gcol + j < g.N) C[j] = f2bf(v[j]);
      }
    } else {
      float* C = (float*)g.C + bz * g.sC + (long)grow * g.ldc + gcol;
      if (EPI == EPI_RES_F32) {
        const float* R = g.R + bz * g.sR + (long)grow * g.ldr + gcol;
        const float* gt = g.gate ? g.gate + (long)(grow / g.rows_per_batch) * g.gate_bstride + gcol : nullptr;
        for (int j = 0; j < 16; ++j) {
          if (gcol + j < g.N) C[j] = R[j] + v[j] * (gt ? gt[j] : 1.0f);
        }
      } else {
        if (full) {
#pragma unroll
          for (int j = 0; j < 4; ++j) *(f32x4*)(C + j * 4) = (f32x4){v[j * 4], v[j * 4 + 1], v[j * 4 + 2], v[j * 4 + 3]};
        } else {
          for (int j = 0; j < 16; ++j) if (gcol + j < g.N) C[j] = v[j];
        }
      }
    }
  }
}

template <int EPI>
int launch(const GemmArgs& g, int batch, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_nt_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    attr = true;
  }
  const int nm = (g.M + BM - 1) / BM, nn = (g.N + BN - 1) / BN;
  hipLaunchKernelGGL(gemm_nt_kernel<EPI>, dim3(nm * nn, 1, batch), dim3(512), LDS_BYTES, st, g);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

}  // namespace

extern "C" int sa_gemm_bf16(const void* A, int64_t lda, int64_t strideA, const void* W, int64_t ldw, int64_t strideW,
                            const float* bias, void* C, int64_t ldc, int64_t strideC, int M, int N, int K, int batch,
                            int epilogue, const float* residual, int64_t ldr, int64_t strideR, const float* gate,
                            int64_t gate_bstride, int rows_per_batch, void* stream) {
  if (!A || !W || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0) return SA_ERR_ARG;
  if (K % BK != 0 || lda % 8 != 0 || ldw % 8 != 0) return SA_ERR_ARG;
  if ((((uintptr_t)A) & 15) || (((uintptr_t)W) & 15)) return SA_ERR_ARG;
  if (epilogue == EPI_RES_F32 && (!residual || (gate && rows_per_batch <= 0))) return SA_ERR_ARG;
  GemmArgs g{(const bf16*)A, lda, strideA, (const bf16*)W, ldw, strideW, bias, C, ldc, strideC,
             residual, ldr, strideR, gate, gate_bstride, rows_per_batch > 0 ? rows_per_batch : 1, M, N, K};
  hipStream_t st = (hipStream_t)stream;
  switch (epilogue) {
    case EPI_BF16: return launch<EPI_BF16>(g, batch, st);
    case EPI_GELU_BF16: return launch<EPI_GELU_BF16>(g, batch, st);
    case EPI_F32: return launch<EPI_F32>(g, batch, st);
    case EPI_RES_F32: return launch<EPI_RES_F32>(g, batch, st);
    case EPI_GELU_ERF_BF16: return launch<EPI_GELU_ERF_BF16>(g, batch, st);
    case EPI_SILU_F32: return launch<EPI_SILU_F32>(g, batch, st);
    default: return SA_ERR_ARG;
  }
}
