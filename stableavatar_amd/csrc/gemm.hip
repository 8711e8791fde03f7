// bf16 "NT" GEMM for every nn.Linear on the StableAvatar DiT / VAE path:
//   C[M,N] = A[M,K] · W[N,K]^T  (+bias, fused epilogue)
// W is the PyTorch Linear weight [out,in] as stored in the checkpoint, so both operands are
// K-contiguous and every MFMA fragment is one 16-byte LDS read.
// Replaces the aten::addmm sites listed in SURVEY.md §2.2 (wan_fantasy_transformer3d_1B.py
// :376-379,550-554,577-578,644-646,832-838,710, vocal_projector_fantasy_1B.py:238-241,313-316).
//
// Two kernels, chosen per call (sa_gemm_bf16_ex; auto = the persistent one wherever it applies):
//  * gemm_s8_kernel: persistent, one wave per SIMD, 256x256 tile, 4 waves x 128x128 with the
//    accumulators in AGPRs, K-tiles of 64 staged by buffer_load...lds into a 2-stage XOR-swizzled
//    LDS ring, the K pipeline running across tile seams (needs K % 128 == 0);
//  * gemm_pp_kernel: 8-wave ping-pong over the same 256x256 tile for any K % 64 == 0
//    (cdna_hip_programming.md §5 "256^2 8-phase template", T3/T4/T5).
// Both use an XCD-aware tile order (T1) and fuse bias / GELU / SiLU / fp32 gated-residual epilogues.
#include <stdlib.h>

#include <utility>

#include "common.h"

namespace {

enum {
  EPI_BF16 = 0, EPI_GELU_BF16 = 1, EPI_F32 = 2, EPI_RES_F32 = 3, EPI_GELU_ERF_BF16 = 4, EPI_SILU_F32 = 5,
  EPI_BF16_T = 6,     // bf16 output stored transposed, C[n * ldc + m]
  EPI_BF16_TP32 = 7   // ... with the rows of each 32-row chunk in the self-attention's P order (its V^T operand,
                      // attention.hip VMODE 1): row 32c + 4q + r at column 32c + 8 (q & 3) + 4 (q >> 2) + r
};

struct GemmArgs {
  const bf16* A; long lda; long sA;
  const bf16* W; long ldw; long sW;
  const float* bias;
  void* C; long ldc; long sC;
  const float* R; long ldr; long sR;     // residual (EPI_RES_F32); may alias C
  const float* gate; long gate_bstride;  // gate[(m / rows_per_batch) * gate_bstride + n]
  int rows_per_batch;
  int M, N, K;
  int group_m;  // tile raster: runs of group_m tile rows, column-major inside a run (L2 reuse per XCD)
  // A in column panels (persistent kernel only): K-tile T (64 columns) lives in panel (T * a_pmul) >> 20,
  // each panel a_pdelta bytes further than contiguous columns would be (a_pmul 0: one plain matrix);
  // a_pextra = the bytes past a tile's rows the buffer range must also cover
  unsigned a_pmul; int a_pdelta; int a_pextra;
};

// flat tile id -> (tile row, tile col): consecutive ids walk down a column of group_m tile rows, then
// the next column, so the 32 tiles one XCD holds at a time (xcd_remap gives it a contiguous id range)
// form a group_m x (32 / group_m) block that shares A rows and W rows in that XCD's L2
__device__ __forceinline__ void tile_coords(int wg, int nm, int nn, int gm, int& mt, int& nt) {
  const int per = gm * nn;
  const int first = (wg / per) * gm;
  const int gsz = min(nm - first, gm);
  const int r = wg % per;
  mt = first + r % gsz;
  nt = r / gsz;
}

constexpr int BM = 256, BN = 256, BK = 64;
// per-FLOP cost of the 192-row persistent tile relative to the 256-row one (auto tile choice; measured r3t2)
// the persistent kernel's K schedule under auto: 9 = three barriers per K step (in the bench clip, 4 sampling
// steps: QKV / cross-Q 520 -> 507 us, O-proj / cross-O / FFN-down 740 -> 702 us average, FFN-up 1594 -> 1549 us,
// bit-identical; profiles/r04/README.md), 8 = the round-3 one-barrier step
#ifndef SA_GEMM_SCHED_DEFAULT
#define SA_GEMM_SCHED_DEFAULT 9
#endif
#ifndef SA_T192_COST
#define SA_T192_COST 1.06  // QKV 1.025, O-proj 1.087, cross-Q 1.05, FFN-up 1.023, FFN-down 1.095 at M = 64 512
#endif
constexpr int HALF_BYTES = 128 * BK * 2;        // 16 KB
constexpr int STAGE_BYTES = 4 * HALF_BYTES;     // 64 KB: A0 A1 B0 B1
constexpr int LDS_BYTES = 2 * STAGE_BYTES;      // 128 KB

// byte offset of 16-byte chunk c of row r in a [rows][64] bf16 tile (128-B rows)
__device__ __forceinline__ int swz128(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// Output store cache policy of the persistent kernels' epilogues (A/B builds: -DSA_STORE_POLICY=<aux>, the
// buffer-store cache-policy bits, gfx950: 1 sc0, 2 nt, 16 sc1).  -1 (default): bf16 rows non-temporal, fp32 plain.
// sc1 stores leave no copy in the XCD's L2 (MI355X_MICROARCH.md store table), so a tile's output burst does not
// evict the K-slices the XCD's other tiles are still reading.
// measurement builds only (scripts/build_variant.sh): 1 = the bf16 row epilogue forms its 16-byte values but does
// not store them (the LDS-strip round trip and the conversion kept; outputs incomplete)
#ifndef SA_EPI_EXP
#define SA_EPI_EXP 0
#endif
// bf16 row epilogue of the persistent kernels: 1 = straight from the accumulators, two column groups' 4-column pieces
// joined into 16-byte row pieces by v_permlane16_swap (s7_bf16_perm_epilogue), the tile's bias loaded at the top of
// its K loop; 0 = the round-4 LDS-strip transposition (also the fallback for a partial last column tile)
#ifndef SA_EPI_V2
#define SA_EPI_V2 1
#endif
#ifndef SA_STORE_POLICY
#define SA_STORE_POLICY -1
#endif
template <class T>
__device__ __forceinline__ void store16(T* base_uniform, long elem_off, u32x4 v) {
  if constexpr (SA_STORE_POLICY < 0) {
    *(u32x4*)(base_uniform + elem_off) = v;
  } else {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base_uniform, (short)0, -1, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(elem_off * (long)sizeof(T)), 0, SA_STORE_POLICY);
  }
}

// apply the epilogue to NC consecutive columns of one output row and store them
template <int EPI, int NC, bool BIAS = true>
__device__ __forceinline__ void epi_row(const GemmArgs& g, float* v, long bz, int grow, int gcol) {
  const bool full = (gcol + NC <= g.N);
  if (BIAS && g.bias) {
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
  if constexpr (EPI == EPI_GELU_BF16 && NC % 2 == 0) {
    // pairs: the bf16 rounding of the Linear output (one v_cvt_pk per pair), then the packed GELU
#pragma unroll
    for (int j = 0; j < NC; j += 2) {
      const bf16x2 h = __builtin_convertvector((f32x2){v[j], v[j + 1]}, bf16x2);
      const f32x2 y = gelu_tanh2(__builtin_convertvector(h, f32x2));
      v[j] = y[0];
      v[j + 1] = y[1];
    }
  } else {
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      // the reference's nn.Linear returns bf16 under autocast; GELU and the gated residual
      // (1B:677-678,688-690) consume that rounded value
      if (EPI == EPI_GELU_BF16 || EPI == EPI_GELU_ERF_BF16 || EPI == EPI_RES_F32) v[j] = bf2f(f2bf(v[j]));
      if (EPI == EPI_GELU_BF16) v[j] = gelu_tanh(v[j]);
      if (EPI == EPI_GELU_ERF_BF16) v[j] = gelu_erf(v[j]);
      if (EPI == EPI_SILU_F32) v[j] = silu(v[j]);
    }
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
          // non-temporal 16-byte stores (global_store ... nt): the epilogue's store burst drains faster
          // (isolated: cross-Q 0.238 vs 0.286 ms, QKV 0.833 vs 0.873, FFN-up 1.535 vs 1.632; in the
          // 30-layer forward 0.4-0.8 % -- the consumers then read more of it from HBM; profiles/r03 r3n)
          if constexpr (SA_EPI_EXP == 1)  // measurement build: the value is formed, not stored
            asm volatile("" ::"v"(__builtin_bit_cast(u32x4, o)));
          else if constexpr (SA_STORE_POLICY < 0)
            __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), (u32x4*)(C + 8 * h));
          else
            store16((bf16*)g.C + bz * g.sC, (long)grow * g.ldc + gcol + 8 * h, __builtin_bit_cast(u32x4, o));
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
// ping-pong kernel (cdna_hip_programming.md "The 256² 8-phase template"): same tile, waves and
// quadrant phases (one block quadrant A_i x B_j per phase), but every phase is {ds_read the phase's fragments, issue one
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
  int mt, nt;
  tile_coords(wg, nm, nn, g.group_m, mt, nt);
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
            if constexpr (EPI == EPI_GELU_BF16 || EPI == EPI_GELU_ERF_BF16 || EPI == EPI_RES_F32)
              t = bf2f(f2bf(t));  // bf16 Linear output, as epi_row
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
// persistent one-wave-per-SIMD kernel (4 waves, 2x2, 128x128 per wave, 256 accumulators in AGPRs; the
// structure hipBLASLt's MT256x256x64 kernel has on gfx950, with our own schedule).  MFMAs and LDS
// reads are inline asm (cdna_hip_programming.md §5.7): hipcc keeps them in program order, the
// accumulators stay in AGPRs ("+a") and the fragment waits are explicit.  Operands are swapped in the
// MFMA (C^T = W·A^T) so each lane holds 4 consecutive output columns of one row.
template <int OFF>
__device__ __forceinline__ void s4_ds(u32x4& d, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}
// TR (EPI_BF16_T): operands in the natural order (C = A·W^T), so each lane holds 4 consecutive output ROWS of one
// column -- 4 consecutive elements of a row of C^T
template <bool TR = false>
__device__ __forceinline__ void s4_mma(f32x4& c, const u32x4& w, const u32x4& x) {
  if constexpr (TR)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(x), "v"(w) : "memory");
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(w), "v"(x) : "memory");
}
template <int MI = 8>
__device__ __forceinline__ void s4_wait_frags(u32x4 (&a)[8], u32x4 (&b)[8]) {
  if constexpr (MI == 8)
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]));
  else
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]));
  asm volatile("" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]));
}

// K-tiles of 64 (128-B rows, so every 1-KB DMA piece is 8 whole cache lines) in a 2-stage LDS ring
// (64 KB per stage: A 256 rows, W 256 rows).  Step t (stage t&1), fragments of (t, k 0-31) already in
// registers: half 0 = 64 MFMAs with the 16 reads of (t, k 32-63) in its first 32; vmcnt(0) + one
// barrier; half 1 = 64 MFMAs with the 16 reads of (t+1, k 0-31) and the 16 DMA pieces of tile t+2
// (into stage t&1) spread over all 8 MFMA rows.
constexpr int S5_STAGE = 2 * 256 * 128;  // 64 KB
constexpr int S5_LDS = 2 * S5_STAGE;     // 128 KB

struct S5Ctx {
  __amdgpu_buffer_rsrc_t ra, rw;
  int aoff[8], woff[8];
  uint32_t lds_dma;          // wave-uniform LDS address of piece 0 (stage 0)
  uint32_t ard[2][2], wrd[2][2];  // [stage][k half] per-lane fragment read bases
};

// MI = A fragments (16-row groups) per wave: 8 for the 256-row tile, 6 for the 192-row one (the A region of a
// stage keeps its 256-row size; a 192-row tile uses the first 24 KB of it).  Pieces 0..MI-1 are A, then 8 of W
template <int STAGE, int PIECE, int MI = 8>
__device__ __forceinline__ void s5_dma(const S5Ctx& c, int ks, int ksa) {
  if constexpr (PIECE < MI) {
    constexpr int i = PIECE;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(c.ra, LDS_PTR((uintptr_t)(c.lds_dma + STAGE * S5_STAGE + i * 4096)), 16,
                                             c.aoff[i], ksa, 0, 0);
  } else {
    constexpr int i = PIECE - MI;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        c.rw, LDS_PTR((uintptr_t)(c.lds_dma + STAGE * S5_STAGE + 256 * 128 + i * 4096)), 16, c.woff[i], ks, 0, 0);
  }
}

template <int STAGE, int KH, int R, int MI = 8>
__device__ __forceinline__ void s5_read(const S5Ctx& c, u32x4 (&a)[8], u32x4 (&b)[8]) {
  if constexpr (R < MI)
    s4_ds<R * 2048>(a[R], c.ard[STAGE][KH]);
  else if constexpr (R < MI + 8)
    s4_ds<(R - MI) * 2048>(b[R - MI], c.wrd[STAGE][KH]);
}

// one 64-MFMA half: MFMA row Q uses (ac[Q], bc[0..7]); the first 4 rows carry the reads of the
// next fragments (stage RS, k half RK) and, when DMA, 4 DMA pieces each of tile ks into stage DS
// DMA piece placement inside a half: packed (4 per MFMA row in rows 0-3) or SPREAD (2 per row, all 8)
// (MI = 6: the 14 pieces as 2 per MFMA row plus one more in rows 0-1)
template <int DS, int Q, int POS, bool DMA, bool SPREAD, int MI = 8>
__device__ __forceinline__ void s5_dma_at(const S5Ctx& c, int ks, int ksa) {
  if constexpr (DMA) {
    if constexpr (SPREAD) {
      if constexpr (POS & 1)
        s5_dma<DS, 2 * Q + (POS >> 1), MI>(c, ks, ksa);
      else if constexpr (POS == 2 && Q < 8 - MI)
        s5_dma<DS, 2 * MI + Q, MI>(c, ks, ksa);
    } else if constexpr (Q < 4) {
      s5_dma<DS, 4 * Q + POS, MI>(c, ks, ksa);
    }
  }
}

template <int RS, int RK, bool DMA, int DS, bool SPREAD = false, int MI = 8, bool TR = false>
__device__ __forceinline__ void s5_half(const S5Ctx& c, f32x4 (&acc)[8][8], u32x4 (&ac)[8], u32x4 (&bc)[8],
                                        u32x4 (&an)[8], u32x4 (&bn)[8], int ks, int ksa) {
#define SA_S5_ROW(Q)                                                                        \
  if constexpr (Q < MI) {                                                                   \
    s4_mma<TR>(acc[Q][0], bc[0], ac[Q]); s4_mma<TR>(acc[Q][1], bc[1], ac[Q]);               \
    if constexpr (Q < 4) { s5_read<RS, RK, 4 * Q, MI>(c, an, bn); }                         \
    s5_dma_at<DS, Q, 0, DMA, SPREAD, MI>(c, ks, ksa);                                       \
    s4_mma<TR>(acc[Q][2], bc[2], ac[Q]); s4_mma<TR>(acc[Q][3], bc[3], ac[Q]);               \
    if constexpr (Q < 4) { s5_read<RS, RK, 4 * Q + 1, MI>(c, an, bn); }                     \
    s5_dma_at<DS, Q, 1, DMA, SPREAD, MI>(c, ks, ksa);                                       \
    s4_mma<TR>(acc[Q][4], bc[4], ac[Q]); s4_mma<TR>(acc[Q][5], bc[5], ac[Q]);               \
    if constexpr (Q < 4) { s5_read<RS, RK, 4 * Q + 2, MI>(c, an, bn); }                     \
    s5_dma_at<DS, Q, 2, DMA, SPREAD, MI>(c, ks, ksa);                                       \
    s4_mma<TR>(acc[Q][6], bc[6], ac[Q]); s4_mma<TR>(acc[Q][7], bc[7], ac[Q]);               \
    if constexpr (Q < 4) { s5_read<RS, RK, 4 * Q + 3, MI>(c, an, bn); }                     \
    s5_dma_at<DS, Q, 3, DMA, SPREAD, MI>(c, ks, ksa);                                       \
  }
  SA_S5_ROW(0) SA_S5_ROW(1) SA_S5_ROW(2) SA_S5_ROW(3) SA_S5_ROW(4) SA_S5_ROW(5) SA_S5_ROW(6) SA_S5_ROW(7)
#undef SA_S5_ROW
}

// persistence: one workgroup per CU walks output tiles u = blockIdx.x + k*gridDim.x and the K
// pipeline runs on across tile seams; the epilogue of tile u runs from a private LDS strip (the
// 4 x 4.3 KB above the 128-KB ring).  Rows past M / N read as zeros from the buffer range check
// (num_records), so the per-lane load offsets are the same for every tile.
constexpr int S7_STRIP = 16 * 68 * 4;             // [16 rows][64 (+4) cols] fp32 per wave
constexpr int S7_LDS = S5_LDS + 4 * S7_STRIP;     // 145 KB

// fp32-output epilogue of an interior tile (gated residual, plain f32, SiLU) straight from the accumulators:
// lane (fr, fc) of wave (wm, wn) holds, in acc[i][j], row m0 + wm*128 + i*16 + fr, columns n0 + wn*128 +
// j*16 + fc*4 + 0..3, so each (i, j) is one 16-byte store per lane with no LDS round trip.  Walked column
// group j outer, row block i inner (step s = 8 j + i): the bias (and the tile's gate row, TILE_GATE) of
// column group j is loaded two groups ahead, the residual (and the per-row gate) AH steps ahead.  a0/b0
// hold the next tile's first fragments here, which caps AH.  Measured against the LDS-strip path (same
// box, interleaved, profiles/r02/gemm_epilogue_study.md): O-proj 0.440 vs 0.447 ms, FFN-down 1.474 vs
// 1.486 ms, 30-layer DiT forward 396.7 vs 398.7 ms; for bf16 outputs the strip path's 16-byte row
// segments stay faster (QKV 0.80 vs 0.94 ms), so those keep it.
template <int EPI, bool TILE_GATE, int MI = 8>
__device__ __forceinline__ void s7_f32_epilogue(const GemmArgs& g, f32x4 (&acc)[8][8], int wm, int wn, int fr, int fc,
                                                int m0, int n0, long bz) {
  constexpr bool RES = EPI == EPI_RES_F32;
  constexpr bool PER_ROW_GATE = RES && !TILE_GATE;
  constexpr int AH = RES ? (PER_ROW_GATE ? 4 : 8) : 1;
  const int col = n0 + wn * 128 + fc * 4;  // + j * 16
  const int row0 = m0 + wm * 16 * MI + fr;  // + i * 16
  const float* tgate = (TILE_GATE && RES && g.gate) ? g.gate + (long)(m0 / g.rows_per_batch) * g.gate_bstride : nullptr;
  f32x4 bj[3], gj[3], rb[AH], gb[PER_ROW_GATE ? AH : 1];
  auto fetch_col = [&](int j) {
    bj[j % 3] = g.bias ? *(const f32x4*)(g.bias + col + j * 16) : (f32x4){0.f, 0.f, 0.f, 0.f};
    if constexpr (RES && TILE_GATE) gj[j % 3] = tgate ? *(const f32x4*)(tgate + col + j * 16) : (f32x4){1.f, 1.f, 1.f, 1.f};
  };
  auto fetch = [&](int st) {
    const int i = st % MI, j = st / MI;
    if constexpr (RES) rb[st % AH] = *(const f32x4*)(g.R + bz * g.sR + (long)(row0 + i * 16) * g.ldr + col + j * 16);
    if constexpr (PER_ROW_GATE)
      gb[st % AH] = *(const f32x4*)(g.gate + (long)((row0 + i * 16) / g.rows_per_batch) * g.gate_bstride + col + j * 16);
  };
  fetch_col(0);
  fetch_col(1);
  if constexpr (RES) {
#pragma unroll
    for (int st = 0; st < AH; ++st) fetch(st);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j + 2 < 8) fetch_col(j + 2);
    // one column group at a time: its accumulators are read from the AGPRs only here (keeps the
    // compiler from hoisting all 256 reads into VGPRs) and no store crosses this point
    if constexpr (MI == 8)
      asm volatile("" : "+a"(acc[0][j]), "+a"(acc[1][j]), "+a"(acc[2][j]), "+a"(acc[3][j]), "+a"(acc[4][j]),
                        "+a"(acc[5][j]), "+a"(acc[6][j]), "+a"(acc[7][j])::"memory");
    else
      asm volatile("" : "+a"(acc[0][j]), "+a"(acc[1][j]), "+a"(acc[2][j]), "+a"(acc[3][j]), "+a"(acc[4][j]),
                        "+a"(acc[5][j])::"memory");
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int st = j * MI + i;
      f32x4 v = acc[i][j];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = v[e] + bj[j % 3][e];
        // the reference's nn.Linear returns bf16 under autocast; the gated residual (1B:677-678,688-690)
        // consumes that rounded value
        if constexpr (RES) t = bf2f(f2bf(t));
        if constexpr (EPI == EPI_SILU_F32) t = silu(t);
        if constexpr (RES) t = rb[st % AH][e] + t * (TILE_GATE ? gj[j % 3][e] : gb[PER_ROW_GATE ? st % AH : 0][e]);
        v[e] = t;
      }
      store16((float*)g.C + bz * g.sC, (long)(row0 + i * 16) * g.ldc + col + j * 16, __builtin_bit_cast(u32x4, v));
      if constexpr (RES) {
        if (st + AH < 8 * MI) fetch(st + AH);
      }
    }
  }
}

// EPI_BF16_T: the tile stored transposed, C[n * ldc + m] = bf16(acc + bias[n]).  With the natural-order MFMA (TR)
// lane (fr, fc) of wave (wm, wn) holds in acc[i][j] rows m0 + wm*16*MI + i*16 + 4 fc + 0..3 of column n0 + wn*128 +
// j*16 + fr: one 8-byte store of 4 consecutive elements of row n of C^T per (i, j), no LDS round trip.  Walked
// column group j outer (its bias loaded once), row block i inner.  M % 4 == 0 (launcher), so a 4-row group is
// wholly inside or outside the matrix.
template <int MI = 8, bool P32 = false>
__device__ __forceinline__ void s7_t_epilogue(const GemmArgs& g, f32x4 (&acc)[8][8], int wm, int wn, int fr, int fc,
                                              int m0, int n0, long bz) {
  const int row0 = m0 + wm * 16 * MI + 4 * fc;  // + i * 16
  bf16* const C = (bf16*)g.C + bz * g.sC;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = n0 + wn * 128 + j * 16 + fr;
    const float b = (g.bias && n < g.N) ? g.bias[n] : 0.f;
    if constexpr (MI == 8)
      asm volatile("" : "+a"(acc[0][j]), "+a"(acc[1][j]), "+a"(acc[2][j]), "+a"(acc[3][j]), "+a"(acc[4][j]),
                        "+a"(acc[5][j]), "+a"(acc[6][j]), "+a"(acc[7][j])::"memory");
    else
      asm volatile("" : "+a"(acc[0][j]), "+a"(acc[1][j]), "+a"(acc[2][j]), "+a"(acc[3][j]), "+a"(acc[4][j]),
                        "+a"(acc[5][j])::"memory");
    if constexpr (P32) {
      // P's order puts row 32c + 4 fc + r of the even block at position 32c + 8 fc + r and the same row of the odd
      // block (+16) at 32c + 8 fc + 4 + r (the tile's rows start on a 32-row boundary: m0, 96 and 128 are multiples
      // of 32): one lane's acc[2c][j] and acc[2c + 1][j] fill 8 consecutive positions, one 16-byte store (half the
      // store instructions of the 8-byte form, same bytes)
#pragma unroll
      for (int i = 0; i < MI; i += 2) {
        const int m = row0 + i * 16;
        const f32x4 v = acc[i][j], w = acc[i + 1][j];
        const bf16x8 o = {f2bf(v[0] + b), f2bf(v[1] + b), f2bf(v[2] + b), f2bf(v[3] + b),
                          f2bf(w[0] + b), f2bf(w[1] + b), f2bf(w[2] + b), f2bf(w[3] + b)};
        bf16* p = C + (long)n * g.ldc + (m & ~31) + 8 * fc;
        if (n < g.N) {
          if (m + 16 < g.M) {
            *(u32x4*)p = __builtin_bit_cast(u32x4, o);
          } else if (m < g.M) {
            *(bf16x4*)p = (bf16x4){o[0], o[1], o[2], o[3]};
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = row0 + i * 16;
        const f32x4 v = acc[i][j];
        const bf16x4 o = {f2bf(v[0] + b), f2bf(v[1] + b), f2bf(v[2] + b), f2bf(v[3] + b)};
        if (n < g.N && m < g.M) *(bf16x4*)(C + (long)n * g.ldc + m) = o;
      }
    }
  }
}

template <int EPI, int MI = 8>
__device__ __forceinline__ void s7_epilogue(const GemmArgs& g, f32x4 (&acc)[8][8], char* smem, int wave, int lane,
                                            int m0, int n0, long bz) {
  constexpr int BMT = 32 * MI;  // tile rows
  const int wm = wave >> 1, wn = wave & 1, fr = lane & 15, fc = lane >> 4;
  float* strip = (float*)(smem + S5_LDS + wave * S7_STRIP);
  if constexpr (EPI == EPI_BF16_T || EPI == EPI_BF16_TP32) {
    s7_t_epilogue<MI, EPI == EPI_BF16_TP32>(g, acc, wm, wn, fr, fc, m0, n0, bz);
    return;
  }
  const int er = lane >> 2, ec = (lane & 3) * 16;
  if constexpr (EPI == EPI_RES_F32 || EPI == EPI_F32 || EPI == EPI_SILU_F32) {
    if (m0 + BMT <= g.M && n0 + BN <= g.N) {  // interior tile (wave-uniform)
      if (EPI != EPI_RES_F32 || !g.gate || m0 / g.rows_per_batch == (m0 + BMT - 1) / g.rows_per_batch)
        s7_f32_epilogue<EPI, true, MI>(g, acc, wm, wn, fr, fc, m0, n0, bz);
      else
        s7_f32_epilogue<EPI, false, MI>(g, acc, wm, wn, fr, fc, m0, n0, bz);
      return;
    }
  }
  // the bias of this lane's 32 output columns, loaded once per tile: a global load inside the row loop
  // below would wait (vmcnt retires in order and counts stores) for every store issued before it, i.e.
  // serialise the tile's 16 store bursts
  f32x4 bias4[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int q = 0; q < 4; ++q) bias4[h][q] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (g.bias) {
    const int c0 = n0 + wn * 128 + ec;
    if (n0 + wn * 128 + 128 <= g.N) {  // wave-uniform: all 8 loads issued back to back
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 4; ++q) bias4[h][q] = *(const f32x4*)(g.bias + c0 + h * 64 + 4 * q);
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int c = c0 + h * 64 + 4 * q + e;
            bias4[h][q][e] = c < g.N ? g.bias[c] : 0.f;
          }
    }
  }
  // one wait for them here, before the row loop (otherwise the compiler's wait before their first use
  // inside a non-unrolled loop body is repeated every iteration, behind that iteration's stores)
  asm volatile("" ::"v"(bias4[0][0]), "v"(bias4[0][1]), "v"(bias4[0][2]), "v"(bias4[0][3]), "v"(bias4[1][0]),
               "v"(bias4[1][1]), "v"(bias4[1][2]), "v"(bias4[1][3]));
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int grow = m0 + wm * 16 * MI + i * 16 + er;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int j = 0; j < 4; ++j) *(f32x4*)(strip + fr * 68 + j * 16 + fc * 4) = acc[i][4 * h + j];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 t = *(const f32x4*)(strip + er * 68 + ec + q * 4);
        v[4 * q] = t[0]; v[4 * q + 1] = t[1]; v[4 * q + 2] = t[2]; v[4 * q + 3] = t[3];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int q = 0; q < 4; ++q)  // unconditional (zeros without a bias): one wait for the loads above
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] += bias4[h][q][e];
      const int gcol = n0 + wn * 128 + h * 64 + ec;
      if (grow < g.M && gcol < g.N) epi_row<EPI, 16, false>(g, v, bz, grow, gcol);
    }
  }
}

template <int MI = 8>
__device__ __forceinline__ void s7_tile(const GemmArgs& g, int u, int total, int G, int nm, int nn, int& m0, int& n0,
                                        long& bz, __amdgpu_buffer_rsrc_t& ra, __amdgpu_buffer_rsrc_t& rw) {
  constexpr int BMT = 32 * MI;
  // rounds of G tiles; within a round the XCD remap hands each XCD a contiguous run of tile ids
  const int per = nm * nn;
  const int round = u / G;
  const int nwg = min(G, total - round * G);
  const int w = round * G + xcd_remap(u - round * G, nwg);
  bz = w / per;
  int mt, nt;
  tile_coords(w - (int)bz * per, nm, nn, g.group_m, mt, nt);
  m0 = mt * BMT;
  n0 = nt * BN;
  const int rows_a = min(BMT, g.M - m0), rows_w = min(BN, g.N - n0);
  ra = __builtin_amdgcn_make_buffer_rsrc((void*)(g.A + bz * g.sA + (long)m0 * g.lda), (short)0,
                                         (int)(rows_a * g.lda * 2) + g.a_pextra, 0x00020000);
  rw = __builtin_amdgcn_make_buffer_rsrc((void*)(g.W + bz * g.sW + (long)n0 * g.ldw), (short)0,
                                         (int)(rows_w * g.ldw * 2), 0x00020000);
}

// The bf16 row epilogue's bias for tile column n0 (lane (fr, fc) of wave column wn: columns n0 + wn*128 + J*16 +
// 4 fc + 0..3 for J = 0..7), issued at the top of the tile's K loop by inline-asm buffer loads.  The compiler does
// not track these loads, so it places no wait for them: the first K step's counted vmcnt (which retires every VMEM
// op older than that step's own DMA) does, and the caller marks the registers defined after it.  A compiler-visible
// load here or in the epilogue gets a vmcnt(0), i.e. waits behind the next tile's DMA in flight.  Returns false
// (nothing loaded: the LDS-strip epilogue runs, with its own loads) for a wave whose 128 columns pass N.
__device__ __forceinline__ bool s8_bias_preload(const GemmArgs& g, f32x4 (&b)[8], int n0, int wn, int lane) {
  if (n0 + wn * 128 + 128 > g.N) return false;  // wave-uniform
  if (!g.bias) {                                 // wave-uniform
#pragma unroll
    for (int J = 0; J < 8; ++J) b[J] = (f32x4){0.f, 0.f, 0.f, 0.f};
    return true;
  }
  const uintptr_t base = (uintptr_t)g.bias;
  const u32x4 rs = {(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)base),
                    (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(base >> 32)),
                    (unsigned)__builtin_amdgcn_readfirstlane(g.N * 4), 0x00020000u};
  const int c0 = n0 + wn * 128 + 4 * ((lane >> 4) & 3);
#pragma unroll
  for (int J = 0; J < 8; ++J)
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(b[J]) : "v"((c0 + J * 16) * 4), "s"(rs));
  return true;
}

// 4 outputs of a bf16 row epilogue (bias already added), packed: the Linear's bf16 rounding, then the activation
// (epi_row's order and arithmetic, so the outputs are bit-identical to the strip path's)
template <int EPI>
__device__ __forceinline__ u32x2 s7_pack4(f32x4 v) {
  if constexpr (EPI == EPI_GELU_BF16) {
    const f32x2 y0 = gelu_tanh2(__builtin_convertvector(__builtin_convertvector((f32x2){v[0], v[1]}, bf16x2), f32x2));
    const f32x2 y1 = gelu_tanh2(__builtin_convertvector(__builtin_convertvector((f32x2){v[2], v[3]}, bf16x2), f32x2));
    v = (f32x4){y0[0], y0[1], y1[0], y1[1]};
  } else if constexpr (EPI == EPI_GELU_ERF_BF16) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = gelu_erf(bf2f(f2bf(v[e])));
  }
  return __builtin_bit_cast(u32x2, (bf16x4){f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])});
}

// bf16 row epilogue straight from the accumulators (interior columns; rows past M not stored).  Lane (fr, fc) holds in
// acc[i][J] row m0 + wm*16*MI + i*16 + fr, columns n0 + wn*128 + J*16 + 4 fc + 0..3.  For a column-group pair (J, J+1)
// two v_permlane16_swap (lanes l <-> l ^ 16, i.e. fc ^ 1) give lane fc = 0 / 2 columns J*16 + 0..7 / 8..15 and lane
// fc = 1 / 3 columns (J+1)*16 + 0..7 / 8..15: one non-temporal 16-byte store per lane, 64 contiguous bytes per row per
// instruction, 32 stores per wave per tile (the strip path's count) and no LDS round trip.  The strip path moved
// 512 KB of fp32 through the LDS per tile (~11 k cycles at the config-2 QKV shape; profiles/r05 gemm stamps).
template <int EPI, int MI>
__device__ __forceinline__ void s7_bf16_perm_epilogue(const GemmArgs& g, f32x4 (&acc)[8][8], const f32x4 (&bj)[8],
                                                      int wm, int wn, int fr, int fc, int m0, int n0, long bz) {
  const int row0 = m0 + wm * 16 * MI + fr;
  bf16* const C = (bf16*)g.C + bz * g.sC + n0 + wn * 128 + (fc & 1) * 16 + (fc >> 1) * 8;
#pragma unroll
  for (int J = 0; J < 8; J += 2) {
    if constexpr (MI == 8)
      asm volatile("" : "+a"(acc[0][J]), "+a"(acc[1][J]), "+a"(acc[2][J]), "+a"(acc[3][J]), "+a"(acc[4][J]),
                        "+a"(acc[5][J]), "+a"(acc[6][J]), "+a"(acc[7][J]), "+a"(acc[0][J + 1]), "+a"(acc[1][J + 1]),
                        "+a"(acc[2][J + 1]), "+a"(acc[3][J + 1]), "+a"(acc[4][J + 1]), "+a"(acc[5][J + 1]),
                        "+a"(acc[6][J + 1]), "+a"(acc[7][J + 1])::"memory");
    else
      asm volatile("" : "+a"(acc[0][J]), "+a"(acc[1][J]), "+a"(acc[2][J]), "+a"(acc[3][J]), "+a"(acc[4][J]),
                        "+a"(acc[5][J]), "+a"(acc[0][J + 1]), "+a"(acc[1][J + 1]), "+a"(acc[2][J + 1]),
                        "+a"(acc[3][J + 1]), "+a"(acc[4][J + 1]), "+a"(acc[5][J + 1])::"memory");
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const f32x4 a = acc[i][J], b = acc[i][J + 1];
      const u32x2 x = s7_pack4<EPI>((f32x4){a[0] + bj[J][0], a[1] + bj[J][1], a[2] + bj[J][2], a[3] + bj[J][3]});
      const u32x2 y = s7_pack4<EPI>(
          (f32x4){b[0] + bj[J + 1][0], b[1] + bj[J + 1][1], b[2] + bj[J + 1][2], b[3] + bj[J + 1][3]});
      const auto r0 = __builtin_amdgcn_permlane16_swap(x[0], y[0], false, false);
      const auto r1 = __builtin_amdgcn_permlane16_swap(x[1], y[1], false, false);
      const u32x4 out = {r0[0], r1[0], r0[1], r1[1]};
      const int row = row0 + i * 16;
      if (row < g.M) __builtin_nontemporal_store(out, (u32x4*)(C + (long)row * g.ldc + J * 16));
    }
  }
}


// ------------------------------------------------------------------------------------------------
// s8 kernel: s7's persistence (tile walk u = blockIdx.x + k*gridDim.x, K pipeline running across tile
// seams, epilogue from a private strip above the ring) on the spread-DMA feed of variant 14: in the
// last two K steps of a tile the DMA fetches K-tiles 0 and 1 of the next tile and the last step's
// fragment reads take its first fragments, so a tile starts with no prologue.
// A's byte offset of K-tile ks / 128 (column panels: see GemmArgs)
template <bool PANEL>
__device__ __forceinline__ int s8_ksa(const GemmArgs& g, int ks) {
  if constexpr (PANEL) return ks + (int)(((unsigned)(ks >> 7) * g.a_pmul) >> 20) * g.a_pdelta;
  return ks;
}

template <int S, bool PANEL, int MI = 8, bool TR = false>
__device__ __forceinline__ void s8_step(const GemmArgs& g, const S5Ctx& c, f32x4 (&acc)[8][8], u32x4 (&a0)[8],
                                        u32x4 (&b0)[8], u32x4 (&a1)[8], u32x4 (&b1)[8], int ks) {
  s4_wait_frags<MI>(a0, b0);
  s5_half<S, 1, false, 0, false, MI, TR>(c, acc, a0, b0, a1, b1, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  s4_wait_frags<MI>(a1, b1);
  __builtin_amdgcn_s_barrier();
  s5_half<S ^ 1, 0, true, S, true, MI, TR>(c, acc, a1, b1, a0, b0, ks, s8_ksa<PANEL>(g, ks));
}

// ------------------------------------------------------------------------------------------------
// s9 K step: the same stage / tile / fragment geometry as s8 on a three-barrier schedule, so the DMA of a K-tile
// gets ~1.5 steps to land (s8: 0.5-1) and the one wait per step is a counted vmcnt, never 0.  Step t (stage S,
// a0/b0 = (t, k 0-31) fragments, read at the end of step t-1), MFMA slots 0 .. 2*NS-1 (NS = 8*MI per k half,
// row-major over (A fragment, W fragment)):
//   slots  0-15  kh0 rows 0-1, reads of A (t, k 32-63) into a1              -> lgkmcnt(0), barrier #1
//   slots 16-39  kh0 rows 2-4, reads of W (t, k 32-63) into b1 and the MI A
//                DMA pieces of tile t+2 (into stage S's A region: its A reads are done)   -> lgkmcnt(0), barrier #2
//   slots 40-T3  the 8 W DMA pieces of tile t+2 (stage S's W region)       -> vmcnt(MI+8): tile t+1 landed, barrier #3
//   slots T3-..  the last 3 kh1 rows, reads of (t+1, k 0-31) into b0 / a0 from stage S^1
// (T3 = 2*NS - 24).  Every fragment register is rewritten >= 12 MFMAs after its last use.
template <int MI>
struct S9 {
  static constexpr int NS = 8 * MI, TOT = 2 * NS, T3 = TOT - 24, NR = 8 + MI;
  // action after MFMA slot s: 0 none, 1+i read a1[i], 9+i read b1[i], 17+i A DMA i, 25+i W DMA i, 33+i read b0[i],
  // 41+i read a0[i]
  static constexpr int act(int s) {
    if (s < 16) return (s & 1) && (s >> 1) < MI ? 1 + (s >> 1) : 0;
    if (s < 40) {
      const int k = (s - 16) / 3, r = (s - 16) % 3;
      if (r == 0) return 9 + k;
      if (r == 1 && k < MI) return 17 + k;
      return 0;
    }
    if (s < T3) {
      const int span = T3 - 40, step = span / 8;
      const int o = s - 40 - step / 2;
      return (o >= 0 && o % step == 0 && o / step < 8) ? 25 + o / step : 0;
    }
    // NR reads over the last 24 slots: b0[0..7] first, then a0[0..MI-1]
    for (int k = 0; k < NR; ++k)
      if (s == T3 + (k * 24) / NR) return k < 8 ? 33 + k : 41 + (k - 8);
    return 0;
  }
};

template <int STAGE_R, int STAGE_D, int MI, int S, bool TR = false>
__device__ __forceinline__ void s9_slot(const S5Ctx& c, f32x4 (&acc)[8][8], u32x4 (&a0)[8], u32x4 (&b0)[8],
                                        u32x4 (&a1)[8], u32x4 (&b1)[8], int ks, int ksa) {
  using P = S9<MI>;
  constexpr int kh = S / P::NS, r = S % P::NS, Q = r / 8, j = r % 8;
  if constexpr (kh == 0)
    s4_mma<TR>(acc[Q][j], b0[j], a0[Q]);
  else
    s4_mma<TR>(acc[Q][j], b1[j], a1[Q]);
  constexpr int a = P::act(S);
  // reads of the current tile's second k half come from stage STAGE_R; the next tile's first half from STAGE_R ^ 1
  if constexpr (a >= 1 && a < 9)
    s4_ds<(a - 1) * 2048>(a1[a - 1], c.ard[STAGE_R][1]);
  else if constexpr (a >= 9 && a < 17)
    s4_ds<(a - 9) * 2048>(b1[a - 9], c.wrd[STAGE_R][1]);
  else if constexpr (a >= 17 && a < 25)
    s5_dma<STAGE_D, a - 17, MI>(c, ks, ksa);
  else if constexpr (a >= 25 && a < 33)
    s5_dma<STAGE_D, MI + a - 25, MI>(c, ks, ksa);
  else if constexpr (a >= 33 && a < 41)
    s4_ds<(a - 33) * 2048>(b0[a - 33], c.wrd[STAGE_R ^ 1][0]);
  else if constexpr (a >= 41)
    s4_ds<(a - 41) * 2048>(a0[a - 41], c.ard[STAGE_R ^ 1][0]);
  if constexpr (S == 15 || S == 39) {
    if constexpr (S == 15)
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a1[0]), "+v"(a1[1]), "+v"(a1[2]), "+v"(a1[3]), "+v"(a1[4]),
                   "+v"(a1[5]), "+v"(a1[6]), "+v"(a1[7])::"memory");
    else
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b1[0]), "+v"(b1[1]), "+v"(b1[2]), "+v"(b1[3]), "+v"(b1[4]),
                   "+v"(b1[5]), "+v"(b1[6]), "+v"(b1[7])::"memory");
    __builtin_amdgcn_s_barrier();
  }
  if constexpr (S == P::T3 - 1) {
    if constexpr (MI == 8)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
}

template <int STAGE, int MI, bool TR, int... Ss>
__device__ __forceinline__ void s9_slots(const S5Ctx& c, f32x4 (&acc)[8][8], u32x4 (&a0)[8], u32x4 (&b0)[8],
                                         u32x4 (&a1)[8], u32x4 (&b1)[8], int ks, int ksa,
                                         std::integer_sequence<int, Ss...>) {
  (s9_slot<STAGE, STAGE, MI, Ss, TR>(c, acc, a0, b0, a1, b1, ks, ksa), ...);
}

// step on the K-tile in stage S; ks = the K-tile (x 128 B) the step's DMA fetches into stage S
template <int S, bool PANEL, int MI = 8, bool TR = false>
__device__ __forceinline__ void s9_step(const GemmArgs& g, const S5Ctx& c, f32x4 (&acc)[8][8], u32x4 (&a0)[8],
                                        u32x4 (&b0)[8], u32x4 (&a1)[8], u32x4 (&b1)[8], int ks) {
  s4_wait_frags<MI>(a0, b0);
  s9_slots<S, MI, TR>(c, acc, a0, b0, a1, b1, ks, s8_ksa<PANEL>(g, ks), std::make_integer_sequence<int, S9<MI>::TOT>{});
}

// MI = 6: 192 x 256 tiles (4 waves x 96 x 128), for launches whose 256-row tile count leaves the last round over
// the CUs mostly empty (the per-rank GEMMs of sequence parallelism: 8 064 rows at N = 8 fill 0.74 of a round of
// 256 x 256 tiles, 0.98 of a round of 192 x 256)
// NOEPI (measurement only, kernels 8 / 9 of sa_gemm_bf16_ex): the tile walk and K loop without the epilogue
template <int EPI, bool PANEL = false, int MI = 8, int SCHED = 8, bool NOEPI = false>
__global__ __launch_bounds__(256, 1) void gemm_s8_kernel(GemmArgs g, int batch) {
  constexpr int BMT = 32 * MI;
  constexpr bool TR = EPI == EPI_BF16_T || EPI == EPI_BF16_TP32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nm = (g.M + BMT - 1) / BMT, nn = (g.N + BN - 1) / BN;
  const int total = nm * nn * batch, G = gridDim.x;
  int u = blockIdx.x;
  S5Ctx c;
  int m0, n0;
  long bz;
  s7_tile<MI>(g, u, total, G, nm, nn, m0, n0, bz, c.ra, c.rw);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = (i * 4 + wave) * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    c.aoff[i] = row * (int)g.lda * 2 + chunk * 16;
    c.woff[i] = row * (int)g.ldw * 2 + chunk * 16;
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(smem);
  c.lds_dma = __builtin_amdgcn_readfirstlane(lds0 + wave * 1024);
  const int fr = lane & 15, fc = lane >> 4;
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int sw = ((4 * kh + fc) ^ ((fr >> 1) & 7)) << 4;
      c.ard[st][kh] = lds0 + st * S5_STAGE + (wm * 16 * MI + fr) * 128 + sw;
      c.wrd[st][kh] = lds0 + st * S5_STAGE + 256 * 128 + (wn * 128 + fr) * 128 + sw;
    }
  const int nk = g.K / 64;  // even (launcher: K % 128 == 0)

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  u32x4 a0[8], b0[8], a1[8], b1[8];
#define SA_S8_DMA(STAGE, P) \
  if constexpr (P < MI + 8) s5_dma<STAGE, P, MI>(c, ks, ksa);
#define SA_S8_DMA_ALL(STAGE, T)                                                                       \
  {                                                                                                   \
    const int ks = (T) * 128, ksa = s8_ksa<PANEL>(g, ks);                                                  \
    SA_S8_DMA(STAGE, 0) SA_S8_DMA(STAGE, 1) SA_S8_DMA(STAGE, 2) SA_S8_DMA(STAGE, 3) SA_S8_DMA(STAGE, 4)   \
    SA_S8_DMA(STAGE, 5) SA_S8_DMA(STAGE, 6) SA_S8_DMA(STAGE, 7) SA_S8_DMA(STAGE, 8) SA_S8_DMA(STAGE, 9)   \
    SA_S8_DMA(STAGE, 10) SA_S8_DMA(STAGE, 11) SA_S8_DMA(STAGE, 12) SA_S8_DMA(STAGE, 13)                   \
    SA_S8_DMA(STAGE, 14) SA_S8_DMA(STAGE, 15)                                                         \
  }
  SA_S8_DMA_ALL(0, 0)
  SA_S8_DMA_ALL(1, 1)
#undef SA_S8_DMA_ALL
#undef SA_S8_DMA
  // K-tile 0 landed; K-tile 1's MI + 8 pieces may still fly
  if constexpr (MI == 8)
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
  static_assert(MI == 8 || MI == 6, "tile rows: 256 or 192");
  __builtin_amdgcn_s_barrier();
  s5_read<0, 0, 0, MI>(c, a0, b0); s5_read<0, 0, 1, MI>(c, a0, b0); s5_read<0, 0, 2, MI>(c, a0, b0);
  s5_read<0, 0, 3, MI>(c, a0, b0); s5_read<0, 0, 4, MI>(c, a0, b0); s5_read<0, 0, 5, MI>(c, a0, b0);
  s5_read<0, 0, 6, MI>(c, a0, b0); s5_read<0, 0, 7, MI>(c, a0, b0); s5_read<0, 0, 8, MI>(c, a0, b0);
  s5_read<0, 0, 9, MI>(c, a0, b0); s5_read<0, 0, 10, MI>(c, a0, b0); s5_read<0, 0, 11, MI>(c, a0, b0);
  s5_read<0, 0, 12, MI>(c, a0, b0); s5_read<0, 0, 13, MI>(c, a0, b0); s5_read<0, 0, 14, MI>(c, a0, b0);
  s5_read<0, 0, 15, MI>(c, a0, b0);

  // the bf16 row epilogues' bias, loaded at the top of each tile (SA_EPI_V2)
  constexpr bool BPRE = SA_EPI_V2 && !NOEPI && !TR && (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_GELU_ERF_BF16);
  f32x4 bpre[8];
  bool pre = false;
  while (true) {
    const int un = u + G;
    const bool has_next = un < total;
    __amdgpu_buffer_rsrc_t cra = c.ra, crw = c.rw, nra = c.ra, nrw = c.rw;
    int nm0 = m0, nn0 = n0;
    long nbz = bz;
    if (has_next) s7_tile<MI>(g, un, total, G, nm, nn, nm0, nn0, nbz, nra, nrw);
    if constexpr (BPRE) pre = s8_bias_preload(g, bpre, n0, wn, lane);
    for (int t = 0; t < nk; t += 2) {
      {
        const bool nx = t + 2 >= nk;  // DMA of the next tile's K-tile t+2-nk (or a re-read of the last)
        c.ra = nx ? nra : cra;
        c.rw = nx ? nrw : crw;
        const int ksd = (nx ? (has_next ? t + 2 - nk : nk - 1) : t + 2) * 128;
        if constexpr (SCHED == 9)
          s9_step<0, PANEL, MI, TR>(g, c, acc, a0, b0, a1, b1, ksd);
        else
          s8_step<0, PANEL, MI, TR>(g, c, acc, a0, b0, a1, b1, ksd);
        if constexpr (BPRE) {  // the bias registers are defined here: the step's counted wait has retired their loads
          if (t == 0)
            asm volatile("" : "+v"(bpre[0]), "+v"(bpre[1]), "+v"(bpre[2]), "+v"(bpre[3]), "+v"(bpre[4]), "+v"(bpre[5]),
                         "+v"(bpre[6]), "+v"(bpre[7]));
        }
      }
      {
        const bool nx = t + 3 >= nk;
        c.ra = nx ? nra : cra;
        c.rw = nx ? nrw : crw;
        const int ksd = (nx ? (has_next ? t + 3 - nk : nk - 1) : t + 3) * 128;
        if constexpr (SCHED == 9)
          s9_step<1, PANEL, MI, TR>(g, c, acc, a0, b0, a1, b1, ksd);
        else
          s8_step<1, PANEL, MI, TR>(g, c, acc, a0, b0, a1, b1, ksd);
      }
    }
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");  // MFMA -> v_accvgpr_read
    if constexpr (BPRE) {
      if (pre)  // two paths: a join would merge the strip path's load waits into this one
        s7_bf16_perm_epilogue<EPI, MI>(g, acc, bpre, wm, wn, lane & 15, lane >> 4, m0, n0, bz);
      else
        s7_epilogue<EPI, MI>(g, acc, smem, wave, lane, m0, n0, bz);
    } else if constexpr (!NOEPI) {
      s7_epilogue<EPI, MI>(g, acc, smem, wave, lane, m0, n0, bz);
    }
    if (!has_next) break;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    u = un;
    m0 = nm0;
    n0 = nn0;
    bz = nbz;
    c.ra = nra;
    c.rw = nrw;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

constexpr int KERNEL_AUTO = 0, KERNEL_PINGPONG = 1, KERNEL_PERSISTENT = 2, KERNEL_PERSISTENT192 = 3;
constexpr int KERNEL_PERSISTENT_AUTO = 4;  // internal: the persistent kernel with the tile rows chosen as by auto
// the s9 (three-barrier) schedule of the persistent kernel: tile rows by auto / 256 / 192
constexpr int KERNEL_S9_AUTO = 5, KERNEL_S9 = 6, KERNEL_S9_192 = 7;
// measurement only: the s9 kernel with the epilogue removed (256- / 192-row tiles), output not written
constexpr int KERNEL_S9_NOEPI = 8, KERNEL_S9_192_NOEPI = 9;
constexpr int KERNEL_MAX = 9;  // (10, the s10 deferred-epilogue kernel, was measured slower and removed: DESIGN.md)

// dynamic-LDS opt-in of one persistent instantiation, once per process
template <int EPI, bool PANEL, int MI, int SCHED, bool NOEPI = false>
void s8_attr() {
  static const bool once = [] {
    (void)hipFuncSetAttribute((const void*)gemm_s8_kernel<EPI, PANEL, MI, SCHED, NOEPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, S7_LDS);
    return true;
  }();
  (void)once;
}

template <int EPI, bool PANEL, int MI, int SCHED, bool NOEPI = false>
void s8_launch(const GemmArgs& g, int batch, dim3 grid, hipStream_t st) {
  s8_attr<EPI, PANEL, MI, SCHED, NOEPI>();
  hipLaunchKernelGGL((gemm_s8_kernel<EPI, PANEL, MI, SCHED, NOEPI>), grid, dim3(256), S7_LDS, st, g, batch);
}

// the persistent schedule auto picks (SA_GEMM_SCHED=8|9 overrides, read once per process)
int env_sched() {
  static const int sc = [] {
    const char* e = getenv("SA_GEMM_SCHED");
    return (e && atoi(e) == 8) ? 8 : (e && atoi(e) == 9) ? 9 : SA_GEMM_SCHED_DEFAULT;
  }();
  return sc;
}

int num_cus() {
  // per device: the persistent grid is one workgroup per CU
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

// the launch-time tile raster override (SA_GEMM_GROUP_M), read once per process
int env_group_m() {
  static const int gm = [] {
    const char* e = getenv("SA_GEMM_GROUP_M");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 0;
  }();
  return gm;
}

template <int EPI>
int launch(const GemmArgs& g_in, int batch, int kernel, hipStream_t st) {
  // one-time per epilogue instantiation: allow the ping-pong kernel's dynamic LDS size
  static const bool attr = [] {
    if constexpr (EPI != EPI_BF16_T && EPI != EPI_BF16_TP32)
      (void)hipFuncSetAttribute((const void*)gemm_pp_kernel<EPI, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                LDS_BYTES);
    return true;
  }();
  (void)attr;
  GemmArgs g = g_in;
  if (kernel == KERNEL_S9_NOEPI || kernel == KERNEL_S9_192_NOEPI) {
    if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_RES_F32) {
      if (g.K % 128 || (long)BM * g.lda * 2 >= 0x7fffffffL || (long)BN * g.ldw * 2 >= 0x7fffffffL) return SA_ERR_ARG;
      if (g.group_m == 0) g.group_m = EPI == EPI_RES_F32 ? 4 : 8;
      const int bmt = kernel == KERNEL_S9_NOEPI ? 256 : 192;
      const int tiles = ((g.M + bmt - 1) / bmt) * ((g.N + BN - 1) / BN) * batch;
      const dim3 grid(min(tiles, num_cus()));
      if (kernel == KERNEL_S9_NOEPI)
        s8_launch<EPI, false, 8, 9, true>(g, batch, grid, st);
      else
        s8_launch<EPI, false, 6, 9, true>(g, batch, grid, st);
      SA_LAUNCH_CHECK();
      return SA_OK;
    }
    return SA_ERR_ARG;
  }
  // auto (measured, profiles/r01/gemm_ab_r4.md): the persistent one-wave-per-SIMD LDS-DMA kernel
  // wherever its K % 128 tiling and 32-bit buffer offsets apply (over the ping-pong: QKV +8-15 %,
  // cross-Q +7-10 %, FFN-up +3-4 %, FFN-down +4 %, O-proj +-1 %), else the ping-pong kernel (e.g. the
  // K = 192 patch embedding)
  const bool persistent_ok = g.K % 128 == 0 && (long)BM * g.lda * 2 < 0x7fffffffL && (long)BN * g.ldw * 2 < 0x7fffffffL;
  const bool s9 = kernel >= KERNEL_S9_AUTO;
  const bool forced = kernel == KERNEL_PERSISTENT || kernel == KERNEL_PERSISTENT192 || kernel == KERNEL_PERSISTENT_AUTO || s9;
  if (forced && !persistent_ok) return SA_ERR_ARG;
  constexpr bool TOUT = EPI == EPI_BF16_T || EPI == EPI_BF16_TP32;
  if constexpr (TOUT) {  // the transposed store exists in the persistent kernel only
    if (!persistent_ok || kernel == KERNEL_PINGPONG || g.M % 4 || g.ldc % 4) return SA_ERR_ARG;
    if (g.ldc < (EPI == EPI_BF16_TP32 ? (g.M + 31) / 32 * 32 : g.M)) return SA_ERR_ARG;
    // P32 stores 16-byte pieces of C^T rows
    if (EPI == EPI_BF16_TP32 && (g.ldc % 8 || g.sC % 8 || ((uintptr_t)g.C & 15))) return SA_ERR_ARG;
  }
  const bool persistent = forced || (kernel == KERNEL_AUTO && persistent_ok);
  const int sched = s9 ? 9 : (kernel == KERNEL_PERSISTENT || kernel == KERNEL_PERSISTENT192) ? 8 : env_sched();
  constexpr bool BF16_OUT = EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_GELU_ERF_BF16 || TOUT;
  if (g.group_m == 0) g.group_m = persistent ? (BF16_OUT ? 8 : 4) : (g.N >= 4096 ? 8 : 1);
  const int nn = (g.N + BN - 1) / BN, ncu = num_cus();
  const long n256 = (long)((g.M + 255) / 256) * nn * batch, n192 = (long)((g.M + 191) / 192) * nn * batch;
  // persistent tile rows: 192 where its rounds over the CUs, at 0.75 of a 256-row tile's work and a measured
  // per-FLOP cost of SA_T192_COST, finish first (the per-rank shapes of sequence parallelism)
  bool t192 = kernel == KERNEL_PERSISTENT192 || kernel == KERNEL_S9_192;
  if ((kernel == KERNEL_AUTO || kernel == KERNEL_PERSISTENT_AUTO || kernel == KERNEL_S9_AUTO) && persistent)
    t192 = (double)((n192 + ncu - 1) / ncu) * 0.75 * SA_T192_COST < (double)((n256 + ncu - 1) / ncu);
  const int nm = t192 ? (g.M + 191) / 192 : (g.M + BM - 1) / BM;
  const dim3 pgrid(min(nm * nn * batch, ncu));
  if (g.a_pmul) {  // column-panel A: the O-projection of the sequence-parallel path only
    if constexpr (EPI == EPI_RES_F32) {
      if (t192)
        sched == 9 ? s8_launch<EPI, true, 6, 9>(g, batch, pgrid, st) : s8_launch<EPI, true, 6, 8>(g, batch, pgrid, st);
      else
        sched == 9 ? s8_launch<EPI, true, 8, 9>(g, batch, pgrid, st) : s8_launch<EPI, true, 8, 8>(g, batch, pgrid, st);
    } else {
      return SA_ERR_ARG;
    }
  } else if (TOUT) {
    if (t192)
      sched == 9 ? s8_launch<EPI, false, 6, 9>(g, batch, pgrid, st) : s8_launch<EPI, false, 6, 8>(g, batch, pgrid, st);
    else
      sched == 9 ? s8_launch<EPI, false, 8, 9>(g, batch, pgrid, st) : s8_launch<EPI, false, 8, 8>(g, batch, pgrid, st);
  } else if (persistent && t192) {
    sched == 9 ? s8_launch<EPI, false, 6, 9>(g, batch, pgrid, st) : s8_launch<EPI, false, 6, 8>(g, batch, pgrid, st);
  } else if (persistent) {
    sched == 9 ? s8_launch<EPI, false, 8, 9>(g, batch, pgrid, st) : s8_launch<EPI, false, 8, 8>(g, batch, pgrid, st);
  } else if constexpr (!TOUT) {
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, true>), dim3(nm * nn, 1, batch), dim3(512), LDS_BYTES, st, g);
  }
  SA_LAUNCH_CHECK();
  return SA_OK;
}

}  // namespace

// a_panel_cols > 0: A is a_panel_cols-wide column panels a_panel_stride elements apart (lda = the panel
// row stride), i.e. A[m, k] = A[(k / a_panel_cols) * a_panel_stride + m * lda + k % a_panel_cols] -- the
// receive layout of the sequence-parallel head exchange, read by the O-projection in place (persistent
// kernel only: a_panel_cols % 64 == 0, one panel per 64-column K-tile)
extern "C" int sa_gemm_bf16_panels(const void* A, int64_t lda, int64_t strideA, const void* W, int64_t ldw,
                                   int64_t strideW, const float* bias, void* C, int64_t ldc, int64_t strideC, int M,
                                   int N, int K, int batch, int epilogue, const float* residual, int64_t ldr,
                                   int64_t strideR, const float* gate, int64_t gate_bstride, int rows_per_batch,
                                   int kernel, int group_m, int64_t a_panel_cols, int64_t a_panel_stride,
                                   void* stream) {
  if (!A || !W || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0) return SA_ERR_ARG;
  if (K % BK != 0 || lda % 8 != 0 || ldw % 8 != 0) return SA_ERR_ARG;
  if ((((uintptr_t)A) & 15) || (((uintptr_t)W) & 15)) return SA_ERR_ARG;
  if (epilogue == EPI_RES_F32 && (!residual || (gate && rows_per_batch <= 0))) return SA_ERR_ARG;
  if (kernel < KERNEL_AUTO || kernel > KERNEL_MAX || kernel == KERNEL_PERSISTENT_AUTO || group_m < 0) return SA_ERR_ARG;
  GemmArgs g{(const bf16*)A, lda, strideA, (const bf16*)W, ldw, strideW, bias, C, ldc, strideC,
             residual, ldr, strideR, gate, gate_bstride, rows_per_batch > 0 ? rows_per_batch : 1, M, N, K,
             group_m > 0 ? group_m : env_group_m(), 0u, 0, 0};
  if (a_panel_cols > 0) {
    // panel p of K-tile T: (T * pmul) >> 20 == T / tpp for every T < K / 64 (checked), bytes in 32 bits
    const long tpp = a_panel_cols / 64, np = (K + a_panel_cols - 1) / a_panel_cols;
    if (a_panel_cols % 64 || lda < a_panel_cols || a_panel_stride < (long)M * lda || batch != 1 || K / 64 > 4096)
      return SA_ERR_ARG;
    if (kernel == KERNEL_PINGPONG) return SA_ERR_ARG;
    const unsigned pmul = (unsigned)(((1L << 20) + tpp - 1) / tpp);
    for (long T = 0; T < K / 64; ++T)
      if ((long)((T * pmul) >> 20) != T / tpp) return SA_ERR_ARG;
    const long delta = (a_panel_stride - a_panel_cols) * 2, extra = (np - 1) * a_panel_stride * 2;
    if (delta >= 0x7fffffffL || extra + (long)BM * lda * 2 >= 0x7fffffffL) return SA_ERR_ARG;
    g.a_pmul = pmul;
    g.a_pdelta = (int)delta;
    g.a_pextra = (int)extra;
    if (kernel == KERNEL_AUTO) kernel = KERNEL_PERSISTENT_AUTO;  // persistent, tile rows by the rounds model
  }
  hipStream_t st = (hipStream_t)stream;
  switch (epilogue) {
    case EPI_BF16: return launch<EPI_BF16>(g, batch, kernel, st);
    case EPI_GELU_BF16: return launch<EPI_GELU_BF16>(g, batch, kernel, st);
    case EPI_F32: return launch<EPI_F32>(g, batch, kernel, st);
    case EPI_RES_F32: return launch<EPI_RES_F32>(g, batch, kernel, st);
    case EPI_GELU_ERF_BF16: return launch<EPI_GELU_ERF_BF16>(g, batch, kernel, st);
    case EPI_SILU_F32: return launch<EPI_SILU_F32>(g, batch, kernel, st);
    case EPI_BF16_T: return launch<EPI_BF16_T>(g, batch, kernel, st);
    case EPI_BF16_TP32: return launch<EPI_BF16_TP32>(g, batch, kernel, st);
    default: return SA_ERR_ARG;
  }
}

// rows past the last panel's row M - 1 that the column-panel O-projection may read (its last tile's full height:
// the panel offset travels in soffset, outside the buffer range check) -- callers size their slack from this
extern "C" int sa_gemm_panel_slack_rows(void) { return BM; }

extern "C" int sa_gemm_bf16_ex(const void* A, int64_t lda, int64_t strideA, const void* W, int64_t ldw,
                               int64_t strideW, const float* bias, void* C, int64_t ldc, int64_t strideC, int M, int N,
                               int K, int batch, int epilogue, const float* residual, int64_t ldr, int64_t strideR,
                               const float* gate, int64_t gate_bstride, int rows_per_batch, int kernel, int group_m,
                               void* stream) {
  return sa_gemm_bf16_panels(A, lda, strideA, W, ldw, strideW, bias, C, ldc, strideC, M, N, K, batch, epilogue,
                             residual, ldr, strideR, gate, gate_bstride, rows_per_batch, kernel, group_m, 0, 0, stream);
}

extern "C" int sa_gemm_bf16(const void* A, int64_t lda, int64_t strideA, const void* W, int64_t ldw, int64_t strideW,
                            const float* bias, void* C, int64_t ldc, int64_t strideC, int M, int N, int K, int batch,
                            int epilogue, const float* residual, int64_t ldr, int64_t strideR, const float* gate,
                            int64_t gate_bstride, int rows_per_batch, void* stream) {
  return sa_gemm_bf16_ex(A, lda, strideA, W, ldw, strideW, bias, C, ldc, strideC, M, N, K, batch, epilogue, residual,
                         ldr, strideR, gate, gate_bstride, rows_per_batch, KERNEL_AUTO, 0, stream);
}
