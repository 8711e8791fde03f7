// bf16 "NT" GEMM for every nn.Linear on the StableAvatar DiT / VAE path:
//   C[M,N] = A[M,K] · W[N,K]^T  (+bias, fused epilogue)
// W is the PyTorch Linear weight [out,in] as stored in the checkpoint, so both operands are
// K-contiguous and every MFMA fragment is one 16-byte LDS read.
// Replaces the aten::addmm sites listed in SURVEY.md §2.2 (wan_fantasy_transformer3d_1B.py
// :376-379,550-554,577-578,644-646,832-838,710, vocal_projector_fantasy_1B.py:238-241,313-316).
//
// Main kernel (gemm_phased_kernel): 256x256 block tile, BK = 64, 8 waves, mfma_f32_16x16x32_bf16.
// Each K-tile is split into four 128x64 half-tiles {A0, A1, B0, B1} staged by global_load_lds into
// a 2-deep LDS ring (XOR-swizzled 128-B rows, source-side swizzle, lane-linear LDS image).  A K-tile is
// computed in four phases, one block-quadrant (A_i x B_j) per phase, each wave owning a 64x32
// sub-tile of every quadrant; each phase issues the next K-tile's half-tile for the slot it frees,
// so three half-tiles stay in flight across the raw s_barrier and the wait is a counted vmcnt(6)
// (cdna_hip_programming.md §5 "256^2 8-phase template", T3/T4/T5).  XCD-aware block order (T1).
#include <stdlib.h>

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
constexpr int HALF_BYTES = 128 * BK * 2;        // 16 KB
constexpr int STAGE_BYTES = 4 * HALF_BYTES;     // 64 KB: A0 A1 B0 B1
constexpr int LDS_BYTES = 2 * STAGE_BYTES;      // 128 KB

// byte offset of 16-byte chunk c of row r in a [rows][64] bf16 tile (128-B rows)
__device__ __forceinline__ int swz128(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// apply the epilogue to NC consecutive columns of one output row and store them
template <int EPI, int NC>
__device__ __forceinline__ void epi_row(const GemmArgs& g, float* v, long bz, int grow, int gcol) {
  const bool full = (gcol + NC <= g.N);
  if (g.bias) {
    if (full) {
#pragma unroll
      for (int j = 0; j < NC / 4; ++j) {
        const f32x4 b = *(const f32x4*)(g.bias + gcol + 4 * j);
        v[4 * j] += b[0]; v[4 * j + 1] += b[1]; v[4 * j + 2] += b[2]; v[4 * j + 3] += b[3];
      }
    } else {
      for (int j = 0; j < NC; ++j) v[j] += (gcol + j < g.N) ? g.bias[gcol + j] : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    if (EPI == EPI_GELU_BF16) v[j] = gelu_tanh(v[j]);
    if (EPI == EPI_GELU_ERF_BF16) v[j] = gelu_erf(v[j]);
    if (EPI == EPI_SILU_F32) v[j] = silu(v[j]);
  }
  if (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_GELU_ERF_BF16) {
    bf16* C = (bf16*)g.C + bz * g.sC + (long)grow * g.ldc + gcol;
    if (full) {
      if constexpr (NC % 8 == 0) {
#pragma unroll
        for (int h = 0; h < NC / 8; ++h) {
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = f2bf(v[8 * h + j]);
          *(bf16x8*)(C + 8 * h) = o;
        }
      } else {
#pragma unroll
        for (int h = 0; h < NC / 4; ++h)
          *(bf16x4*)(C + 4 * h) = (bf16x4){f2bf(v[4 * h]), f2bf(v[4 * h + 1]), f2bf(v[4 * h + 2]), f2bf(v[4 * h + 3])};
      }
    } else {
      for (int j = 0; j < NC; ++j) if (gcol + j < g.N) C[j] = f2bf(v[j]);
    }
  } else {
    float* C = (float*)g.C + bz * g.sC + (long)grow * g.ldc + gcol;
    if (EPI == EPI_RES_F32) {
      const float* R = g.R + bz * g.sR + (long)grow * g.ldr + gcol;
      const float* gt = g.gate ? g.gate + (long)(grow / g.rows_per_batch) * g.gate_bstride + gcol : nullptr;
      if (full) {
#pragma unroll
        for (int j = 0; j < NC / 4; ++j) {
          const f32x4 r = *(const f32x4*)(R + 4 * j);
          const f32x4 gg = gt ? *(const f32x4*)(gt + 4 * j) : (f32x4){1.f, 1.f, 1.f, 1.f};
          *(f32x4*)(C + 4 * j) = (f32x4){r[0] + v[4 * j] * gg[0], r[1] + v[4 * j + 1] * gg[1],
                                         r[2] + v[4 * j + 2] * gg[2], r[3] + v[4 * j + 3] * gg[3]};
        }
      } else {
        for (int j = 0; j < NC; ++j)
          if (gcol + j < g.N) C[j] = R[j] + v[j] * (gt ? gt[j] : 1.0f);
      }
    } else {
      if (full) {
#pragma unroll
        for (int j = 0; j < NC / 4; ++j) *(f32x4*)(C + 4 * j) = (f32x4){v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]};
      } else {
        for (int j = 0; j < NC; ++j) if (gcol + j < g.N) C[j] = v[j];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// phased kernel

template <int EPI>
__global__ __launch_bounds__(512) void gemm_phased_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qm = wave >> 2, qn = wave & 3;  // this wave's 64x32 sub-tile inside each 128x128 quadrant
  const int nm = (g.M + BM - 1) / BM, nn = (g.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, nm * nn);
  const int mt = wg / nn, nt = wg % nn;
  const int m0 = mt * BM, n0 = nt * BN;
  const long bz = blockIdx.z;
  const bf16* A = g.A + bz * g.sA;
  const bf16* W = g.W + bz * g.sW;

  // staging: half-tile h in {0:A0, 1:A1, 2:B0, 3:B1}; 2 glds per thread per half-tile
  long goff[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = i * 8 + wave;
      const int row = j * 8 + (lane >> 3);
      const int chunk = (lane & 7) ^ ((row >> 1) & 7);
      if (h < 2) {
        const int r = min(m0 + h * 128 + row, g.M - 1);
        goff[h][i] = (long)r * g.lda + chunk * 8;
      } else {
        const int r = min(n0 + (h - 2) * 128 + row, g.N - 1);
        goff[h][i] = (long)r * g.ldw + chunk * 8;
      }
    }
  auto issue = [&](int h, int kt, int buf) {
    const long k0 = (long)kt * BK;
    const bf16* base = h < 2 ? A : W;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = i * 8 + wave;
      __builtin_amdgcn_global_load_lds((const void*)(base + goff[h][i] + k0),
                                       LDS_PTR(smem + buf * STAGE_BYTES + h * HALF_BYTES + j * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[4][4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) acc[q][m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // phase p reads quadrant (A_i, B_j): p0 (A0,B0) p1 (A0,B1) p2 (A1,B1) p3 (A1,B0);
  // it issues the next K-tile's half-tile in order A0, B0, B1, A1 (the slot freed earliest first)
  const int nk = g.K / BK;
  issue(0, 0, 0);
  issue(2, 0, 0);
  issue(3, 0, 0);
  issue(1, 0, 0);
  bf16x8 a[4][2], b0[2][2], b1[2][2];
  const int c0 = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool nxt = kt + 1 < nk;
    const char* S = smem + cur * STAGE_BYTES;
#define SA_PHASE_WAIT(VN, VL)                                          \
  if (nxt) asm volatile("s_waitcnt vmcnt(" #VN ")" ::: "memory");     \
  else asm volatile("s_waitcnt vmcnt(" #VL ")" ::: "memory");          \
  __builtin_amdgcn_s_barrier();                                        \
  asm volatile("" ::: "memory");
    // ---- phase 0: A0 x B0
    if (nxt) issue(0, kt + 1, cur ^ 1);
    SA_PHASE_WAIT(6, 4)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) a[m][kk] = *(const bf16x8*)(S + 0 * HALF_BYTES + swz128(qm * 64 + m * 16 + (lane & 15), kk * 4 + c0));
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) b0[n][kk] = *(const bf16x8*)(S + 2 * HALF_BYTES + swz128(qn * 32 + n * 16 + (lane & 15), kk * 4 + c0));
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[0][m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][kk], b0[n][kk], acc[0][m][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    // ---- phase 1: A0 x B1
    if (nxt) issue(2, kt + 1, cur ^ 1);
    SA_PHASE_WAIT(6, 2)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) b1[n][kk] = *(const bf16x8*)(S + 3 * HALF_BYTES + swz128(qn * 32 + n * 16 + (lane & 15), kk * 4 + c0));
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[1][m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][kk], b1[n][kk], acc[1][m][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    // ---- phase 2: A1 x B1
    if (nxt) issue(3, kt + 1, cur ^ 1);
    SA_PHASE_WAIT(6, 0)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) a[m][kk] = *(const bf16x8*)(S + 1 * HALF_BYTES + swz128(qm * 64 + m * 16 + (lane & 15), kk * 4 + c0));
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[2][m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][kk], b1[n][kk], acc[2][m][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    // ---- phase 3: A1 x B0 (operands already in registers)
    if (nxt) issue(1, kt + 1, cur ^ 1);
    SA_PHASE_WAIT(8, 0)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[3][m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][kk], b0[n][kk], acc[3][m][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
#undef SA_PHASE_WAIT
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue: per wave and per (quadrant, m-tile) a 16x32 fp32 strip through LDS; 8 columns per lane
  float* strip = (float*)(smem + wave * (16 * 36 * 4));
  const int er = lane >> 2, ec = (lane & 3) * 8;
  const int qa[4] = {0, 0, 1, 1}, qb[4] = {0, 1, 1, 0};
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) strip[((lane >> 4) * 4 + i) * 36 + n * 16 + (lane & 15)] = acc[q][m][n][i];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      float v[8];
      const f32x4 t0 = *(const f32x4*)(strip + er * 36 + ec);
      const f32x4 t1 = *(const f32x4*)(strip + er * 36 + ec + 4);
      v[0] = t0[0]; v[1] = t0[1]; v[2] = t0[2]; v[3] = t0[3];
      v[4] = t1[0]; v[5] = t1[1]; v[6] = t1[2]; v[7] = t1[3];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const int grow = m0 + qa[q] * 128 + qm * 64 + m * 16 + er;
      const int gcol = n0 + qb[q] * 128 + qn * 32 + ec;
      if (grow < g.M && gcol < g.N) epi_row<EPI, 8>(g, v, bz, grow, gcol);
    }
}

// ------------------------------------------------------------------------------------------------
// ping-pong kernel (cdna_hip_programming.md "The 256² 8-phase template"): same tile, waves and
// quadrant phases as gemm_phased_kernel, but every phase is {ds_read the phase's fragments, issue one
// half-tile, counted vmcnt} barrier {16 MFMAs} barrier, and waves 4-7 run one barrier behind waves
// 0-3, so on each SIMD one wave reads while its partner multiplies.  Two K-tiles per iteration
// (E = 2i in buffer 0, O = 2i+1 in buffer 1); phase ph issues, in order,
//   A1(O) | A0(E+2) B0(E+2) B1(E+2) A1(E+2) | A0(O+2) B0(O+2) B1(O+2)
// so every half-tile is read >= 6 phases after it is issued: vmcnt(10) (5 half-tiles of 2 glds
// still in flight) before each phase's first barrier retires whatever the next phase reads.  Each
// slot is restaged >= 2 phases after its last read, except A0 (1 phase), whose reads are retired by
// an lgkmcnt(0) before the reading phase's first barrier.
// DIRECT: operands swapped in the MFMA (C^T = W·A^T), so each lane holds 4 consecutive output
// columns of one row and the epilogue stores straight from the accumulators (no LDS transpose).
template <int EPI, bool DIRECT>
__global__ __launch_bounds__(512) void gemm_pp_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qm = wave >> 2, qn = wave & 3;
  const bool g1 = qm == 1;
  const int nm = (g.M + BM - 1) / BM, nn = (g.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, nm * nn);
  const int mt = wg / nn, nt = wg % nn;
  const int m0 = mt * BM, n0 = nt * BN;
  const long bz = blockIdx.z;
  const bf16* A = g.A + bz * g.sA;
  const bf16* W = g.W + bz * g.sW;
  const int nk = g.K / BK;

  long goff[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = i * 8 + wave;
      const int row = j * 8 + (lane >> 3);
      const int chunk = (lane & 7) ^ ((row >> 1) & 7);
      if (h < 2) {
        const int r = min(m0 + h * 128 + row, g.M - 1);
        goff[h][i] = (long)r * g.lda + chunk * 8;
      } else {
        const int r = min(n0 + (h - 2) * 128 + row, g.N - 1);
        goff[h][i] = (long)r * g.ldw + chunk * 8;
      }
    }
  // half-tile h: 0 = A0, 1 = A1, 2 = B0, 3 = B1
  auto issue = [&](int h, int kt) {
    if (kt >= nk) return;
    const long k0 = (long)kt * BK;
    const bf16* base = h < 2 ? A : W;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = i * 8 + wave;
      __builtin_amdgcn_global_load_lds((const void*)(base + goff[h][i] + k0),
                                       LDS_PTR(smem + (kt & 1) * STAGE_BYTES + h * HALF_BYTES + j * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[4][4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) acc[q][m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue = phases 1..7 of iteration -1
  issue(0, 0); issue(2, 0); issue(3, 0); issue(1, 0);
  issue(0, 1); issue(2, 1); issue(3, 1);
  if (nk >= 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (g1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  bf16x8 a[4][2], b0[2][2], b1[2][2];
  const int c0 = lane >> 4;
  auto read_a = [&](const char* S, int half) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        a[m][kk] = *(const bf16x8*)(S + half * HALF_BYTES + swz128(qm * 64 + m * 16 + (lane & 15), kk * 4 + c0));
  };
  auto read_b = [&](bf16x8 (&b)[2][2], const char* S, int half) {
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        b[n][kk] = *(const bf16x8*)(S + (2 + half) * HALF_BYTES + swz128(qn * 32 + n * 16 + (lane & 15), kk * 4 + c0));
  };
  auto mma = [&](f32x4 (&c)[4][2], const bf16x8 (&b)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          if constexpr (DIRECT)
            c[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[n][kk], a[m][kk], c[m][n], 0, 0, 0);
          else
            c[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][kk], b[n][kk], c[m][n], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
  };
#define SA_PP_MID(FULL)                                                   \
  if (FULL) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");             \
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                   \
  __builtin_amdgcn_s_barrier();                                           \
  __builtin_amdgcn_sched_barrier(0);
#define SA_PP_END()                                                       \
  __builtin_amdgcn_sched_barrier(0);                                      \
  __builtin_amdgcn_s_barrier();                                           \
  __builtin_amdgcn_sched_barrier(0);

  const int iters = (nk + 1) / 2;
  for (int it = 0; it < iters; ++it) {
    const int E = 2 * it, O = E + 1;
    const bool full = O + 2 < nk;
    const bool has_o = O < nk;
    const char* S0 = smem;
    const char* S1 = smem + STAGE_BYTES;
    // ph0: A0 x B0 of E
    read_a(S0, 0);
    read_b(b0, S0, 0);
    issue(1, O);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    SA_PP_MID(full)
    mma(acc[0], b0);
    SA_PP_END()
    // ph1: A0 x B1
    read_b(b1, S0, 1);
    issue(0, E + 2);
    SA_PP_MID(full)
    mma(acc[1], b1);
    SA_PP_END()
    // ph2: A1 x B1
    read_a(S0, 1);
    issue(2, E + 2);
    SA_PP_MID(full)
    mma(acc[2], b1);
    SA_PP_END()
    // ph3: A1 x B0
    issue(3, E + 2);
    SA_PP_MID(full)
    mma(acc[3], b0);
    SA_PP_END()
    // ph4..7: the same on O (buffer 1)
    if (has_o) {
      read_a(S1, 0);
      read_b(b0, S1, 0);
    }
    issue(1, E + 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    SA_PP_MID(full)
    if (has_o) mma(acc[0], b0);
    SA_PP_END()
    if (has_o) read_b(b1, S1, 1);
    issue(0, O + 2);
    SA_PP_MID(full)
    if (has_o) mma(acc[1], b1);
    SA_PP_END()
    if (has_o) read_a(S1, 1);
    issue(2, O + 2);
    SA_PP_MID(full)
    if (has_o) mma(acc[2], b1);
    SA_PP_END()
    issue(3, O + 2);
    SA_PP_MID(full)
    if (has_o) mma(acc[3], b0);
    SA_PP_END()
  }
#undef SA_PP_MID
#undef SA_PP_END
  if (!g1) __builtin_amdgcn_s_barrier();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (DIRECT) {
    // per quadrant: issue every residual / gate / bias load of its 8 fragments first, then combine and
    // store (R may alias C element-for-element, so loads of a fragment must precede its store)
    const int qa[4] = {0, 0, 1, 1}, qb[4] = {0, 1, 1, 0};
    constexpr bool RES = EPI == EPI_RES_F32;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rb = m0 + qa[q] * 128 + qm * 64 + (lane & 15);
      const int cb = n0 + qb[q] * 128 + qn * 32 + (lane >> 4) * 4;
      f32x4 bv[2], rv[4][2], gv[4][2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int c = cb + n * 16;
        bv[n] = (g.bias && c + 4 <= g.N) ? *(const f32x4*)(g.bias + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const int row = rb + m * 16, c = cb + n * 16;
          const bool ok = row < g.M && c + 4 <= g.N;
          rv[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};
          gv[m][n] = (f32x4){1.f, 1.f, 1.f, 1.f};
          if (RES && ok) {
            rv[m][n] = *(const f32x4*)(g.R + bz * g.sR + (long)row * g.ldr + c);
            if (g.gate) gv[m][n] = *(const f32x4*)(g.gate + (long)(row / g.rows_per_batch) * g.gate_bstride + c);
          }
        }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const int row = rb + m * 16, c = cb + n * 16;
          if (row >= g.M || c >= g.N) continue;
          if (c + 4 > g.N) {  // ragged right edge: element-wise path
            float v[4] = {acc[q][m][n][0], acc[q][m][n][1], acc[q][m][n][2], acc[q][m][n][3]};
            epi_row<EPI, 4>(g, v, bz, row, c);
            continue;
          }
          f32x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float t = acc[q][m][n][i] + bv[n][i];
            if constexpr (EPI == EPI_SILU_F32) t = silu(t);
            if constexpr (EPI == EPI_GELU_BF16) t = gelu_tanh(t);
            if constexpr (EPI == EPI_GELU_ERF_BF16) t = gelu_erf(t);
            o[i] = RES ? rv[m][n][i] + t * gv[m][n][i] : t;
          }
          if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_GELU_ERF_BF16) {
            bf16* C = (bf16*)g.C + bz * g.sC + (long)row * g.ldc + c;
            *(bf16x4*)C = (bf16x4){f2bf(o[0]), f2bf(o[1]), f2bf(o[2]), f2bf(o[3])};
          } else {
            *(f32x4*)((float*)g.C + bz * g.sC + (long)row * g.ldc + c) = o;
          }
        }
    }
    return;
  }
  __syncthreads();

  float* strip = (float*)(smem + wave * (16 * 36 * 4));
  const int er = lane >> 2, ec = (lane & 3) * 8;
  const int qa[4] = {0, 0, 1, 1}, qb[4] = {0, 1, 1, 0};
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) strip[((lane >> 4) * 4 + i) * 36 + n * 16 + (lane & 15)] = acc[q][m][n][i];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      float v[8];
      const f32x4 t0 = *(const f32x4*)(strip + er * 36 + ec);
      const f32x4 t1 = *(const f32x4*)(strip + er * 36 + ec + 4);
      v[0] = t0[0]; v[1] = t0[1]; v[2] = t0[2]; v[3] = t0[3];
      v[4] = t1[0]; v[5] = t1[1]; v[6] = t1[2]; v[7] = t1[3];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const int grow = m0 + qa[q] * 128 + qm * 64 + m * 16 + er;
      const int gcol = n0 + qb[q] * 128 + qn * 32 + ec;
      if (grow < g.M && gcol < g.N) epi_row<EPI, 8>(g, v, bz, grow, gcol);
    }
}

// ------------------------------------------------------------------------------------------------
// w4 kernel: 4 waves x (128x128 per wave), one wave per SIMD with the 256 accumulators in AGPRs.
// K is staged in 32-deep sub-tiles (A 256x32 + B 256x32 = 32 KB) through a 4-slot LDS ring: while
// sub-tile s is multiplied, s+1 is already landed (its fragments are read between the MFMAs of s)
// and s+2, s+3 are in flight -> one barrier per 64 MFMAs/wave and a counted vmcnt(8).
constexpr int W4_SLOT = 2 * 256 * 64;  // A + B sub-tile, 64-B rows
constexpr int W4_LDS = 4 * W4_SLOT;    // 128 KB

__device__ __forceinline__ int swz64(int r, int c) { return r * 64 + ((c ^ ((r >> 1) & 3)) << 4); }

template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nm = (g.M + BM - 1) / BM, nn = (g.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, nm * nn);
  const int mt = wg / nn, nt = wg % nn;
  const int m0 = mt * BM, n0 = nt * BN;
  const long bz = blockIdx.z;
  const bf16* A = g.A + bz * g.sA;
  const bf16* W = g.W + bz * g.sW;

  // staging: per sub-tile each wave issues 4 A + 4 B wave-instructions of 16 rows x 64 B
  long aoff[4], woff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (i * 4 + wave) * 16 + (lane >> 2);
    const int chunk = (lane & 3) ^ ((row >> 1) & 3);
    aoff[i] = (long)min(m0 + row, g.M - 1) * g.lda + chunk * 8;
    woff[i] = (long)min(n0 + row, g.N - 1) * g.ldw + chunk * 8;
  }
  const int ns = g.K / 32;
  auto issue = [&](int s) {
    char* base = smem + (s & 3) * W4_SLOT;
    const long k0 = (long)s * 32;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_global_load_lds((const void*)(A + aoff[i] + k0), LDS_PTR(base + (i * 4 + wave) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(W + woff[i] + k0),
                                       LDS_PTR(base + 256 * 64 + (i * 4 + wave) * 1024), 16, 0, 0);
    }
  };
  auto read = [&](int s, bf16x8 (&a)[8], bf16x8 (&b)[8]) {
    const char* base = smem + (s & 3) * W4_SLOT;
    const int c = lane >> 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = *(const bf16x8*)(base + swz64(wm * 128 + i * 16 + (lane & 15), c));
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = *(const bf16x8*)(base + 256 * 64 + swz64(wn * 128 + j * 16 + (lane & 15), c));
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: sub-tiles 0..2 in flight, wait for 0 and 1
  issue(0);
  if (ns > 1) issue(1);
  if (ns > 2) issue(2);
  if (ns > 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  read(0, a0, b0);
  // sub-tile s+1 must be visible before its fragments are read: own DMA of s+1 retired (s+2, s+3
  // may fly), then the barrier, which also certifies every wave finished reading slot (s+3)&3.
  // (ns is even: K % 64 == 0.)  Reads past the last sub-tile hit a stale slot and are never used.
  for (int s = 0; s < ns; s += 2) {
    if (s + 2 < ns) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + 3 < ns) issue(s + 3);
    read(s + 1, a1, b1);
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], b0[j], acc[i][j], 0, 0, 0);
    if (s + 3 < ns) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + 4 < ns) issue(s + 4);
    read(s + 2, a0, b0);
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1[j], acc[i][j], 0, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue: per wave 16x128 fp32 strips through LDS, 32 columns per lane
  float* strip = (float*)(smem + wave * (16 * 132 * 4));
  const int er = lane >> 2, ec = (lane & 3) * 32;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) strip[((lane >> 4) * 4 + r) * 132 + j * 16 + (lane & 15)] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const int grow = m0 + wm * 128 + i * 16 + er;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 t = *(const f32x4*)(strip + er * 132 + ec + h * 16 + q * 4);
        v[4 * q] = t[0]; v[4 * q + 1] = t[1]; v[4 * q + 2] = t[2]; v[4 * q + 3] = t[3];
      }
      const int gcol = n0 + wn * 128 + ec + h * 16;
      if (grow < g.M && gcol < g.N) epi_row<EPI, 16>(g, v, bz, grow, gcol);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------------------------------------
// v1 kernel (2-phase, kept for A/B measurements: SA_GEMM_V1=1)

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
  long aoff[4], woff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wave * 4 + i) * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
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
      for (int m = 0; m < 8; ++m) a[m] = *(const bf16x8*)(As + swz128(wm * 128 + m * 16 + (lane & 15), c));
#pragma unroll
      for (int n = 0; n < 4; ++n) b[n] = *(const bf16x8*)(Bs + swz128(wn * 64 + n * 16 + (lane & 15), c));
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], b[n], acc[m][n], 0, 0, 0);
    }
  }
  __syncthreads();
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
    if (grow < g.M && gcol < g.N) epi_row<EPI, 16>(g, v, bz, grow, gcol);
  }
}

int g_gemm_variant = -1;  // 0 = v1 (2-phase), 1 = phased (8 waves), 2 = w4 (4 waves, AGPR accumulators),
                          // 3 = ping-pong 8-phase, 4 = ping-pong with direct (operand-swapped) epilogue

template <int EPI>
int launch(const GemmArgs& g, int batch, hipStream_t st) {
  static int attr = 0;
  if (g_gemm_variant < 0) {
    const char* e = getenv("SA_GEMM_VARIANT");
    g_gemm_variant = e ? atoi(e) : 4;
  }
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_nt_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_phased_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_w4_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, W4_LDS);
    (void)hipFuncSetAttribute((const void*)gemm_pp_kernel<EPI, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_pp_kernel<EPI, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES);
    attr = 1;
  }
  const int nm = (g.M + BM - 1) / BM, nn = (g.N + BN - 1) / BN;
  if (g_gemm_variant == 0)
    hipLaunchKernelGGL(gemm_nt_kernel<EPI>, dim3(nm * nn, 1, batch), dim3(512), LDS_BYTES, st, g);
  else if (g_gemm_variant == 1)
    hipLaunchKernelGGL(gemm_phased_kernel<EPI>, dim3(nm * nn, 1, batch), dim3(512), LDS_BYTES, st, g);
  else if (g_gemm_variant == 2)
    hipLaunchKernelGGL(gemm_w4_kernel<EPI>, dim3(nm * nn, 1, batch), dim3(256), W4_LDS, st, g);
  else if (g_gemm_variant == 3) {
    // fp32 outputs store straight from the (operand-swapped) accumulators; bf16 outputs go through
    // the LDS transpose for 16-B row stores
    constexpr bool F32_OUT = EPI == EPI_RES_F32 || EPI == EPI_F32 || EPI == EPI_SILU_F32;
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, F32_OUT>), dim3(nm * nn, 1, batch), dim3(512), LDS_BYTES, st, g);
  }
  else
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, true>), dim3(nm * nn, 1, batch), dim3(512), LDS_BYTES, st, g);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

}  // namespace

extern "C" int sa_gemm_set_variant(int variant) {
  if (variant < 0 || variant > 4) return SA_ERR_ARG;
  g_gemm_variant = variant;
  return SA_OK;
}

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
