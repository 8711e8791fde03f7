// 3-D causal VAE decoder kernels (reference: wan/models/wan_vae.py), whole-clip formulation
// (see oracle/vae.py for why the frame-by-frame causal cache equals whole-clip causal padding).
// Activations are channels-last bf16 [T, H, W, C] so every conv is an implicit GEMM whose
// A-operand rows are contiguous channel vectors.
//  sa_conv3d_cl        : CausalConv3d (wan_vae.py:20-39) / Conv2d 3x3 / 1x1 as implicit GEMM on MFMA
//                        (16x16x32 bf16), fused: nearest-exact 2x upsample of the input (Upsample
//                        :60-66), bias, residual add (ResidualBlock :223 / AttentionBlock :265) and the
//                        time_conv frame interleave of Resample 'upsample3d' (:137-140)
//  sa_vae_rmsnorm_silu : RMS_norm (:42-57) (+SiLU) over channels
//  sa_vae_input        : z / (1/std) + mean  (:553-557) -> channels-last bf16 (channel-padded)
//  sa_vae_output       : channels-last fp32 -> [3, T, H, W] with clamp(-1,1) (:668) (+/2+0.5 clamp(0,1)
//                        of decode_latents, pipeline:427)
//  sa_softmax_rows     : softmax of fp32 score rows -> bf16 P (AttentionBlock SDPA :255-259)
//  sa_transpose_bf16   : batched 2-D transpose (V -> V^T for the P·V GEMM)
#include "common.h"

#include <stdlib.h>

#include <type_traits>

#ifndef SA_CONV_DMA_DEFAULT
#define SA_CONV_DMA_DEFAULT 2
#endif

namespace {

struct ConvArgs {
  const bf16* x;
  int T, H, W, Cin;  // logical input (== output spatial dims)
  int Hin, Win;      // physical input dims (H/2, W/2 when upsampling)
  int upsample;
  const bf16* w;     // [Coutp][kt][kh][kw][Cin]
  const float* bias;
  int Cout, kt, kh, kw;
  const bf16* res;   // [T, H, W, Cout] or null
  void* y;
  int out_f32;
  int ichalf;        // >0: time_conv interleave, out[2t + n/ichalf][h][w][n%ichalf]
  long M;
  int down;          // 0: stride 1; 1: ZeroPad2d((0,1,0,1)) + 3x3 stride 2 (Resample 'downsample*',
                     // :91-100), input [T][Hin][Win]; 2: (3,1,1) time_conv, stride 2, no padding
                     // (:99, :150-157): output frame t reads input frames 2t .. 2t+2
  const bf16* xprev; // causal cache [kt-1][Hin][Win][Cin]: input frames -(kt-1)..-1 (null: zeros)
};

constexpr int BM = 128, BK = 32;

__device__ __forceinline__ int swz64(int r, int c) { return r * 64 + ((c ^ ((r >> 1) & 3)) << 4); }

template <int NT>
__global__ __launch_bounds__(256, 2) void conv3d_cl_kernel(ConvArgs a) {
  constexpr int BN = NT * 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int SBYTES = BM * 64 + BN * 64;  // one stage: A tile then B tile
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long m0 = (long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const long HW = (long)a.H * a.W;
  const int K = a.kt * a.kh * a.kw * a.Cin;
  const int nk = K / BK;

  // this thread's two A staging chunks: rows r = idx>>2, chunk c = idx&3
  int ar[2], ac[2], at[2], ah[2], aw[2];
  bool arow_ok[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = tid + j * 256;
    ar[j] = idx >> 2;
    ac[j] = idx & 3;
    const long m = m0 + ar[j];
    arow_ok[j] = m < a.M;
    const long mm = arow_ok[j] ? m : 0;
    at[j] = mm / HW;
    const int p = mm % HW;
    ah[j] = p / a.W;
    aw[j] = p % a.W;
  }
  constexpr int BCH = BN * 4;  // 16-B chunks of the B tile
  constexpr int BPT = (BCH + 255) / 256;

#ifndef SA_CONV_DEPTH
#define SA_CONV_DEPTH 2
#endif
  // register staging ring: the loads of step ks + 1 are in flight while step ks is stored and multiplied,
  // so a step's loads have a whole step of MFMAs behind them before their LDS write (depth 2, with
  // __launch_bounds__(256, 2) holding the 192-wide tile at 202 VGPRs: decode 283.0 vs 288.4 ms,
  // bit-identical, profiles/r03/README.md r3y)
  constexpr int NS = SA_CONV_DEPTH;
  u32x4 ra[NS][2], rb[NS][BPT];
  // The K loop walks (tap, channel chunk) in order; the A-row source pointers are recomputed only
  // when the tap changes (every Cin/BK steps) and the chunk offset advances in between, so the
  // im2col index arithmetic is off the per-step path (Cin % BK == 0 is checked by the launcher).
  const bf16* asrc[2];
  int ld_tap = 0, ld_ci = 0;
  long ld_k0 = 0;
  auto set_tap = [&](int tap) {
    const int dt = tap / (a.kh * a.kw), dh = (tap / a.kw) % a.kh, dw = tap % a.kw;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int ti, hi, wi;
      bool ok;
      if (a.down == 1) {  // wave-uniform
        ti = at[j];
        hi = 2 * ah[j] + dh;
        wi = 2 * aw[j] + dw;
        ok = arow_ok[j] && hi < a.Hin && wi < a.Win;
      } else if (a.down == 2) {
        ti = 2 * at[j] + dt;
        hi = ah[j];
        wi = aw[j];
        ok = arow_ok[j];
      } else {
        ti = at[j] + dt - (a.kt - 1);
        hi = ah[j] + dh - (a.kh - 1) / 2;
        wi = aw[j] + dw - (a.kw - 1) / 2;
        ok = arow_ok[j] && (ti >= 0 || a.xprev) && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
      }
      asrc[j] = nullptr;
      if (ok) {
        const int hp = a.upsample ? (hi >> 1) : hi, wp = a.upsample ? (wi >> 1) : wi;
        const bf16* xb = a.x;
        if (ti < 0) {  // only with a cache (chunked decode): frame kt-1+ti of the previous chunk's tail
          xb = a.xprev;
          ti += a.kt - 1;
        }
        asrc[j] = xb + (((long)ti * a.Hin + hp) * a.Win + wp) * a.Cin + ac[j] * 8;
      }
    }
  };
  auto load = [&](int s) {  // loads step (ld_tap, ld_ci) into ring slot s and advances to the next one
    if (ld_ci == 0) set_tap(ld_tap);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      ra[s][j] = asrc[j] ? *(const u32x4*)(asrc[j] + ld_ci) : (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int idx = tid + j * 256;
      if (idx < BCH) {
        const int r = idx >> 2, c = idx & 3;
        rb[s][j] = *(const u32x4*)(a.w + (long)(n0 + r) * K + ld_k0 + c * 8);
      }
    }
    ld_k0 += BK;
    ld_ci += BK;
    if (ld_ci == a.Cin) {
      ld_ci = 0;
      ++ld_tap;
    }
  };
  auto store = [&](int buf, int s) {
#pragma unroll
    for (int j = 0; j < 2; ++j) *(u32x4*)(smem + buf * SBYTES + swz64(ar[j], ac[j])) = ra[s][j];
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int idx = tid + j * 256;
      if (idx < BCH) *(u32x4*)(smem + buf * SBYTES + BM * 64 + swz64(idx >> 2, idx & 3)) = rb[s][j];
    }
  };

  // wave tile: WM x WN waves over the BM x BN tile; each wave holds AI 16-row A fragments x NB 16-column
  // B fragments (2 x 2 when NT is even: 4 + NT/2 fragment reads per NT*2 MFMAs instead of 2 + NT)
  constexpr int WN = NT % 2 == 0 ? 2 : 1, WM = 4 / WN;
  constexpr int AI = BM / WM / 16, NB = NT / WN;
  const int wm = wave / WN, wn = wave % WN;
  f32x4 acc[AI][NB];
#pragma unroll
  for (int i = 0; i < AI; ++i)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[i][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // one K step: store slot S of step ks, refill it with step ks + NS, barrier, MFMAs
  auto kstep = [&](int ks, auto sc) {
    constexpr int S = decltype(sc)::value;
    const int buf = ks & 1;
    store(buf, S);
    if (ks + NS < nk) load(S);  // issued before the barrier: the wait at the barrier hides part of its latency
    __syncthreads();
    const int c = lane >> 4;
    bf16x8 af[AI];
#pragma unroll
    for (int i = 0; i < AI; ++i)
      af[i] = *(const bf16x8*)(smem + buf * SBYTES + swz64(wm * AI * 16 + i * 16 + (lane & 15), c));
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const bf16x8 bfr = *(const bf16x8*)(smem + buf * SBYTES + BM * 64 + swz64((wn * NB + n) * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < AI; ++i) acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][n], 0, 0, 0);
    }
  };
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (s < nk) load(s);
  if constexpr (NS == 1) {
    for (int ks = 0; ks < nk; ++ks) kstep(ks, std::integral_constant<int, 0>{});
  } else {
    static_assert(NS == 2, "register ring depth 1 or 2");
    int ks = 0;
    for (; ks + 1 < nk; ks += 2) {
      kstep(ks, std::integral_constant<int, 0>{});
      kstep(ks + 1, std::integral_constant<int, 1>{});
    }
    if (ks < nk) kstep(ks, std::integral_constant<int, 0>{});
  }
  __syncthreads();

  // epilogue through a per-wave 16 x (NB*16) fp32 strip
  constexpr int LD = NB * 16 + 4;
  float* strip = (float*)(smem + wave * 16 * LD * 4);
  const int er = lane >> 2, q = lane & 3;
  constexpr int CPL = NB * 4;  // columns per lane
#pragma unroll
  for (int i = 0; i < AI; ++i) {
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) strip[((lane >> 4) * 4 + r) * LD + n * 16 + (lane & 15)] = acc[i][n][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const long m = m0 + wm * AI * 16 + i * 16 + er;
    if (m < a.M) {
      const long t = m / HW, p = m % HW;
#pragma unroll
      for (int g = 0; g < CPL; g += 4) {
        const int n = n0 + wn * NB * 16 + q * CPL + g;
        if (n < a.Cout) {
          float v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = strip[er * LD + q * CPL + g + u] + a.bias[n + u];
          long off;
          if (a.ichalf > 0) {
            const int half = n / a.ichalf, nc = n % a.ichalf;
            off = ((2 * t + half) * HW + p) * a.ichalf + nc;
          } else {
            off = m * a.Cout + n;
          }
          if (a.res) {
            const bf16x4 rr = *(const bf16x4*)(a.res + off);
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] += bf2f(rr[u]);
          }
          if (a.out_f32) {
            *(f32x4*)((float*)a.y + off) = (f32x4){v[0], v[1], v[2], v[3]};
          } else {
            *(bf16x4*)((bf16*)a.y + off) = (bf16x4){f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
}

template <int NT>
int launch_conv(const ConvArgs& a, hipStream_t st) {
  constexpr int BN = NT * 16;
  const int lds_main = 2 * (BM * 64 + BN * 64);
  const int lds_epi = 4 * 16 * (BN + 4) * 4;
  const int lds = lds_main > lds_epi ? lds_main : lds_epi;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv3d_cl_kernel<NT>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  dim3 grid((unsigned)((a.M + BM - 1) / BM), (a.Cout + BN - 1) / BN);
  hipLaunchKernelGGL(conv3d_cl_kernel<NT>, grid, dim3(256), lds, st, a);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

// conv epilogue through a per-wave 16 x (NB*16) fp32 strip in LDS (the ring is free by now): bias, optional
// residual, time_conv interleave, bf16 or fp32 store
template <int AI, int NB>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, const f32x4 (&acc)[AI][NB], char* smem, long m0,
                                              int n0, long HW, int wm, int wn, int wave, int lane) {
  constexpr int LD = NB * 16 + 4;
  float* strip = (float*)(smem + wave * 16 * LD * 4);
  const int er = lane >> 2, q = lane & 3;
  constexpr int CPL = NB * 4;
#pragma unroll
  for (int i = 0; i < AI; ++i) {
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) strip[((lane >> 4) * 4 + r) * LD + n * 16 + (lane & 15)] = acc[i][n][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const long m = m0 + wm * AI * 16 + i * 16 + er;
    if (m < a.M) {
      const long t = m / HW, p = m % HW;
#pragma unroll
      for (int g = 0; g < CPL; g += 4) {
        const int n = n0 + wn * NB * 16 + q * CPL + g;
        if (n < a.Cout) {
          float v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = strip[er * LD + q * CPL + g + u] + a.bias[n + u];
          long off;
          if (a.ichalf > 0) {
            const int half = n / a.ichalf, nc = n % a.ichalf;
            off = ((2 * t + half) * HW + p) * a.ichalf + nc;
          } else {
            off = m * a.Cout + n;
          }
          if (a.res) {
            const bf16x4 rr = *(const bf16x4*)(a.res + off);
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] += bf2f(rr[u]);
          }
          if (a.out_f32) {
            *(f32x4*)((float*)a.y + off) = (f32x4){v[0], v[1], v[2], v[3]};
          } else {
            *(bf16x4*)((bf16*)a.y + off) = (bf16x4){f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
}

// ---- the same implicit GEMM with both operands staged by LDS-DMA (buffer_load_dwordx4 ... lds) into a
// 3-stage ring instead of through VGPRs and ds_write_b128.  The register-staged kernel above spends the
// LDS store path on 14 KB per K step per workgroup (ds_write_b128: ~13 cycles of the CU's store path per
// wave-instruction, MI355X_MICROARCH.md LDS table) for 48 MFMAs per step at NT = 6.  Here each wave
// issues 1-KB pieces (16 rows x 64 B): lane l loads row 16p + l/4, swizzled chunk (l%4) ^ ((row>>1)&3), so
// the LDS image is the one swz64 reads.  Every (tile, tap) reads ONE input frame (a tile is 128 pixels of
// one frame: the launcher requires H*W % 128 == 0), so a tap's descriptor spans exactly that frame (or the
// causal cache frame, or nothing: num_records 0 reads zeros); padded taps point their lanes out of range.
// Same (tap, channel chunk) K order and the same MFMA sequence per accumulator as conv3d_cl_kernel:
// bit-identical output.  Stride-1 convs only (down == 0).
template <int NT, int BMT, int NSTAGE>
__device__ __forceinline__ void conv3d_dma_body(const ConvArgs& a) {
  constexpr int BN = NT * 16;
  constexpr int APW = BMT / 64;                  // A pieces (16 rows) per wave per step
  constexpr int BPW = (NT + 3) / 4;              // B pieces per wave per step (waves past NT / BPW issue none)
  static_assert(NT % BPW == 0, "a wave holds all or none of its B pieces");
  constexpr int PPS = APW + BPW;                 // DMA instructions per wave per step (B-less waves: APW)
  constexpr int SBYTES = BMT * 64 + 4 * BPW * 1024;  // one stage: A tile then B pieces
  constexpr uint32_t OOR = 0x80000000u;          // out-of-range offset: the load returns zeros
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long m0 = (long)blockIdx.x * BMT;
  const int n0 = blockIdx.y * BN;
  const long HW = (long)a.H * a.W;
  const int K = a.kt * a.kh * a.kw * a.Cin;
  const int nk = K / BK, cpt = a.Cin / BK;
  const int tile_t = (int)(m0 / HW);  // every row of the tile is in this frame
  const long frame_bytes = (long)a.Hin * a.Win * a.Cin * 2;

  // A lanes: pieces APW*w + j -> tile rows r = 16p + lane/4
  int ah[APW], aw[APW];
  uint32_t acol[APW];
  bool aok[APW];
#pragma unroll
  for (int j = 0; j < APW; ++j) {
    const int r = 16 * (APW * wave + j) + (lane >> 2);
    const long m = m0 + r;
    aok[j] = m < a.M;
    const int p = (int)((aok[j] ? m : m0) % HW);
    ah[j] = p / a.W;
    aw[j] = p % a.W;
    acol[j] = (uint32_t)(((lane & 3) ^ ((r >> 1) & 3)) << 4);
  }
  // B lanes: pieces w*BPW + j -> weight rows n0 + 16p + lane/4
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, (int)((long)gridDim.y * BN * K * 2), 0x00020000);
  uint32_t boff[BPW];
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    const int p = wave * BPW + j;
    const int r = 16 * p + (lane >> 2);
    boff[j] = (uint32_t)((long)(n0 + r) * K * 2 + ((((lane & 3) ^ ((r >> 1) & 3))) << 4));
  }
  const bool bw = wave * BPW < NT;  // this wave loads B pieces (wave-uniform)
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));

  // issue side: (tap, channel chunk) of the next step to load, its frame descriptor and A lane offsets
  int ld_tap = -1, ld_ci = 0, ld_ks = 0;
  __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, 0, 0x00020000);
  uint32_t aoff[APW];
#pragma unroll
  for (int j = 0; j < APW; ++j) aoff[j] = OOR;
  auto set_tap = [&](int tap) {
    const int dt = tap / (a.kh * a.kw), dh = (tap / a.kw) % a.kh, dw = tap % a.kw;
    int ti = tile_t + dt - (a.kt - 1);
    const bf16* fb = nullptr;
    if (ti >= 0) {
      fb = a.x + (long)ti * a.Hin * a.Win * a.Cin;
    } else if (a.xprev) {
      fb = a.xprev + (long)(ti + a.kt - 1) * a.Hin * a.Win * a.Cin;
    }
    rx = __builtin_amdgcn_make_buffer_rsrc((void*)(fb ? fb : a.x), (short)0, fb ? (int)frame_bytes : 0, 0x00020000);
#pragma unroll
    for (int j = 0; j < APW; ++j) {
      const int hi = ah[j] + dh - (a.kh - 1) / 2, wi = aw[j] + dw - (a.kw - 1) / 2;
      const bool ok = aok[j] && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
      const int hp = a.upsample ? (hi >> 1) : hi, wp = a.upsample ? (wi >> 1) : wi;
      aoff[j] = ok ? (uint32_t)(((long)hp * a.Win + wp) * a.Cin * 2) + acol[j] : OOR;
    }
  };
  auto issue = [&](int slot) {  // DMA of step ld_ks into ring slot `slot`
    if (ld_ci == 0) set_tap(++ld_tap);
    const uint32_t sb = lds0 + slot * SBYTES;
#pragma unroll
    for (int j = 0; j < APW; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, LDS_PTR((uintptr_t)(sb + (APW * wave + j) * 1024)), 16, aoff[j],
                                               ld_ci * 2, 0, 0);
    if (bw) {
#pragma unroll
      for (int j = 0; j < BPW; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rw, LDS_PTR((uintptr_t)(sb + BMT * 64 + (wave * BPW + j) * 1024)), 16, boff[j], ld_ks * BK * 2, 0, 0);
    }
    ++ld_ks;
    ld_ci += BK;
    if (ld_ci == a.Cin) ld_ci = 0;
  };

  constexpr int WN = NT % 2 == 0 ? 2 : 1, WM = 4 / WN;
  constexpr int AI = BMT / WM / 16, NB = NT / WN;
  const int wm = wave / WN, wn = wave % WN;
  f32x4 acc[AI][NB];
#pragma unroll
  for (int i = 0; i < AI; ++i)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[i][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // steps ks+1 .. ks+NSTAGE-2 in flight while step ks is multiplied
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) issue(s);
  for (int ks = 0; ks < nk; ++ks) {
    // step ks landed: at most the later issued steps' pieces still in flight
    const int ahead = min(nk - 1 - ks, NSTAGE - 2);
    if (ahead >= 2) {
      if (bw)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PPS) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * APW) : "memory");
    } else if (ahead == 1) {
      if (bw)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PPS) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(APW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // into the slot every wave finished reading at step ks - 1
    if (ks + NSTAGE - 1 < nk) issue((ks + NSTAGE - 1) % NSTAGE);
    const char* st = smem + (ks % NSTAGE) * SBYTES;
    const int c = lane >> 4;
    bf16x8 af[AI];
#pragma unroll
    for (int i = 0; i < AI; ++i) af[i] = *(const bf16x8*)(st + swz64(wm * AI * 16 + i * 16 + (lane & 15), c));
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const bf16x8 bfr = *(const bf16x8*)(st + BMT * 64 + swz64((wn * NB + n) * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < AI; ++i) acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][n], 0, 0, 0);
    }
  }
  (void)cpt;
  __syncthreads();
  conv_epilogue<AI, NB>(a, acc, smem, m0, n0, HW, wave / WN, wave % WN, wave, lane);
}

// (the body is a device function: host compilation does not emit the stub of a kernel that declares buffer
// resource variables itself)
template <int NT, int BMT, int NSTAGE>
__global__ __launch_bounds__(256, 2) void conv3d_dma_kernel(ConvArgs a) {
  conv3d_dma_body<NT, BMT, NSTAGE>(a);
}

template <int NT, int BMT, int NSTAGE>
int launch_conv_dma(const ConvArgs& a, hipStream_t st) {
  constexpr int BN = NT * 16, BPW = (NT + 3) / 4;
  const int lds_main = NSTAGE * (BMT * 64 + 4 * BPW * 1024);
  const int lds_epi = 4 * 16 * (BN + 4) * 4;
  const int lds = lds_main > lds_epi ? lds_main : lds_epi;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv3d_dma_kernel<NT, BMT, NSTAGE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              lds);
    attr = true;
  }
  dim3 grid((unsigned)((a.M + BMT - 1) / BMT), (a.Cout + BN - 1) / BN);
  hipLaunchKernelGGL((conv3d_dma_kernel<NT, BMT, NSTAGE>), grid, dim3(256), lds, st, a);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

// SA_CONV_DMA (read per call so a test can compare the paths in one process): 0 the register-staged kernel for
// every conv; 1 the LDS-DMA kernel on 128-row tiles; 2 (default) 256-row tiles where a frame holds them
int conv_dma_enabled() {
  const char* e = getenv("SA_CONV_DMA");
  return e ? atoi(e) : SA_CONV_DMA_DEFAULT;
}

// ---------------------------------------------------------------------------------------------

// rows of C channels; G lanes per row (power of two >= C/8), 64/G rows per wave
template <int G>
__global__ __launch_bounds__(256) void rmsnorm_silu_kernel(const bf16* x, bf16* y, const float* gamma, long rows,
                                                           int C, int do_silu) {
  const int lane = threadIdx.x & 63;
  const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / G) + lane / G;
  const int g = lane % G;
  const bool ok = row < rows && g * 8 < C;
  float v[8];
  float s = 0.f;
  if (ok) {
    const bf16x8 a = *(const bf16x8*)(x + row * C + g * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) { v[j] = bf2f(a[j]); s += v[j] * v[j]; }
  }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  // F.normalize: x / max(||x||, 1e-12), then * sqrt(C) * gamma
  const float inv = sqrtf((float)C) / fmaxf(sqrtf(s), 1e-12f);
  if (ok) {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = v[j] * inv * gamma[g * 8 + j];
      if (do_silu) t = silu(t);
      o[j] = f2bf(t);
    }
    *(bf16x8*)(y + row * C + g * 8) = o;
  }
}

// the same RMS_norm + SiLU for C = 24 Q (96 / 192 / 384: three quarters of rmsnorm_silu_kernel<4Q>'s lanes
// would hold channels, a quarter zeros): Q lanes per row, each holding chunks j, j + Q, j + 2Q, so every lane
// is busy.  The sum of squares is formed in rmsnorm_silu_kernel<4Q>'s exact order -- each 8-channel chunk
// sequentially, then its xor tree, whose first two levels pair chunk j with j + 2Q and then with j + Q (the
// chunks past C are the zeros the tree adds) -- so the output is bit-identical.
template <int Q>
__global__ __launch_bounds__(256) void rmsnorm_silu3_kernel(const bf16* x, bf16* y, const float* gamma, long rows,
                                                             int C, int do_silu) {
  const int lane = threadIdx.x & 63;
  const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / Q) + lane / Q;
  const int j = lane % Q;
  const bool ok = row < rows;
  float v[3][8];
  float c[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    c[k] = 0.f;
    if (ok) {
      const bf16x8 a = *(const bf16x8*)(x + row * C + (j + k * Q) * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) { v[k][e] = bf2f(a[e]); c[k] += v[k][e] * v[k][e]; }
    }
  }
  float s = (c[0] + c[2]) + (c[1] + 0.f);
#pragma unroll
  for (int o = Q / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float inv = sqrtf((float)C) / fmaxf(sqrtf(s), 1e-12f);
  if (ok) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = v[k][e] * inv * gamma[(j + k * Q) * 8 + e];
        if (do_silu) t = silu(t);
        o[e] = f2bf(t);
      }
      *(bf16x8*)(y + row * C + (j + k * Q) * 8) = o;
    }
  }
}

__global__ void vae_input_kernel(const float* z, int Cz, long THW, const float* mean, const float* stdv, bf16* out,
                                 int Cp) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= THW * Cp) return;
  const int c = idx % Cp;
  const long p = idx / Cp;
  float v = 0.f;
  if (c < Cz) v = z[c * THW + p] * stdv[c] + mean[c];
  out[idx] = f2bf(v);
}

__global__ void vae_output_kernel(const float* in, int Cs, int C, long THW, float* out, int post) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= THW * C) return;
  const int c = idx / THW;
  const long p = idx % THW;
  float v = fminf(fmaxf(in[p * Cs + c], -1.f), 1.f);
  if (post) v = fminf(fmaxf(v / 2.f + 0.5f, 0.f), 1.f);
  out[idx] = v;
}

__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* s, long lds_, bf16* p, long ldp, int n,
                                                           float scale) {
  const long row = blockIdx.x;
  const float* sr = s + row * lds_;
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float mx = -INFINITY;
  for (int i = tid; i < n; i += 256) mx = fmaxf(mx, sr[i]);
  mx = wave_max(mx);
  if (lane == 0) red[w] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int i = tid; i < n; i += 256) sum += __expf((sr[i] - mx) * scale);
  sum = wave_sum(sum);
  if (lane == 0) red[w] = sum;
  __syncthreads();
  const float inv = 1.f / (red[0] + red[1] + red[2] + red[3]);
  for (int i = tid; i < n; i += 256) p[row * ldp + i] = f2bf(__expf((sr[i] - mx) * scale) * inv);
}

__global__ void transpose_kernel(const bf16* in, long ldi, long si, bf16* out, long ldo, long so, int R, int Cc) {
  __shared__ bf16 tile[32][33];
  const long z = blockIdx.z;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < Cc) ? in[z * si + (long)r * ldi + c] : f2bf(0.f);
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (c < Cc && r < R) out[z * so + (long)c * ldo + r] = tile[tx][i];
  }
}

// encoder output: channels-last fp32 [THW][C_stride] (mu | log_var) -> [2 Cz][THW] with
// mu normalised as (mu - mean) * (1 / std) (wan_vae.py:538-544); log_var passes through
__global__ void vae_latent_out_kernel(const float* in, int C_stride, int Cz, long THW, const float* mean,
                                      const float* stdv, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= THW * 2 * Cz) return;
  const int c = (int)(i / THW);
  const long p = i % THW;
  const float v = in[p * C_stride + c];
  out[i] = c < Cz ? (v - mean[c]) * (1.0f / stdv[c]) : v;
}

inline unsigned nblk(long n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace

extern "C" int sa_conv3d_cl(const void* x, int T, int H, int W, int Cin, int upsample, const void* w,
                            const float* bias, int Cout, int Cout_pad, int kt, int kh, int kw, const void* residual,
                            void* y, int out_f32, int interleave_half, const void* x_prev, void* stream) {
  if (!x || !w || !bias || !y || T <= 0 || H <= 0 || W <= 0) return SA_ERR_ARG;
  if (Cin % BK || Cout % 4 || (kt != 1 && kt != 3) || (kh != 1 && kh != 3) || (kw != 1 && kw != 3)) return SA_ERR_ARG;
  if (upsample && (H % 2 || W % 2)) return SA_ERR_ARG;
  if (interleave_half > 0 && (Cout != 2 * interleave_half || residual)) return SA_ERR_ARG;
  ConvArgs a{(const bf16*)x, T, H, W, Cin, upsample ? H / 2 : H, upsample ? W / 2 : W, upsample, (const bf16*)w,
             bias, Cout, kt, kh, kw, (const bf16*)residual, y, out_f32, interleave_half, (long)T * H * W, 0,
             kt > 1 ? (const bf16*)x_prev : nullptr};
  hipStream_t st = (hipStream_t)stream;
  // N tile chosen so the packed weight rows (Cout_pad) cover whole tiles
  const int dma = conv_dma_enabled();
  if (dma && ((long)H * W) % BM == 0) {
    // 256-row tiles where a frame holds whole 256-pixel tiles: the 192-wide convs on a 2-stage ring (256 VGPRs,
    // two workgroups per CU), the 96-wide and head convs on a 3-stage ring.  Decode 227 ms vs 239.5 with 128-row
    // 192-wide tiles and 249 with 128-row tiles everywhere (SA_CONV_DMA=1); profiles/r04/README.md
    const bool m256 = dma >= 2 && ((long)H * W) % 256 == 0;
    if (Cout_pad % 192 == 0 && Cout > 96)
      return m256 ? launch_conv_dma<12, 256, 2>(a, st) : launch_conv_dma<12, 128, 3>(a, st);
    if (Cout_pad % 96 == 0 && Cout > 16)  // (a 2-stage ring here: 233.7 ms)
      return m256 ? launch_conv_dma<6, 256, 3>(a, st) : launch_conv_dma<6, 128, 3>(a, st);
    if (Cout_pad % 16 == 0 && Cout <= 16)
      return m256 ? launch_conv_dma<1, 256, 3>(a, st) : launch_conv_dma<1, 128, 3>(a, st);
    return SA_ERR_ARG;
  }
  if (Cout_pad % 192 == 0 && Cout > 96) return launch_conv<12>(a, st);
  if (Cout_pad % 96 == 0 && Cout > 16) return launch_conv<6>(a, st);
  if (Cout_pad % 16 == 0 && Cout <= 16) return launch_conv<1>(a, st);
  return SA_ERR_ARG;
}

extern "C" int sa_conv3d_cl_down(const void* x, int T_out, int H_in, int W_in, int Cin, int mode, const void* w,
                                 const float* bias, int Cout, int Cout_pad, void* y, void* stream) {
  if (!x || !w || !bias || !y || T_out <= 0 || H_in <= 0 || W_in <= 0) return SA_ERR_ARG;
  if (Cin % BK || Cout % 4 || (mode != 1 && mode != 2)) return SA_ERR_ARG;
  if (mode == 1 && (H_in % 2 || W_in % 2)) return SA_ERR_ARG;
  const int H = mode == 1 ? H_in / 2 : H_in, W = mode == 1 ? W_in / 2 : W_in;
  const int kt = mode == 1 ? 1 : 3, kh = mode == 1 ? 3 : 1;
  ConvArgs a{(const bf16*)x, T_out, H, W, Cin, H_in, W_in, 0, (const bf16*)w, bias, Cout, kt, kh, kh,
             nullptr, y, 0, 0, (long)T_out * H * W, mode, nullptr};
  hipStream_t st = (hipStream_t)stream;
  if (Cout_pad % 192 == 0 && Cout > 96) return launch_conv<12>(a, st);
  if (Cout_pad % 96 == 0 && Cout > 16) return launch_conv<6>(a, st);
  return SA_ERR_ARG;
}

extern "C" int sa_vae_rmsnorm_silu(const void* x, void* y, const float* gamma, int64_t rows, int C, int do_silu,
                                   void* stream) {
  if (!x || !y || !gamma || C % 8 || C > 512) return SA_ERR_ARG;
  const int g8 = C / 8;
  hipStream_t st = (hipStream_t)stream;
  const char* e = getenv("SA_RMS3");
  if (!e || atoi(e)) {  // every lane busy for C = 96 / 192 / 384 (bit-identical; SA_RMS3=0 for the A/B)
    if (C == 96) {
      hipLaunchKernelGGL(rmsnorm_silu3_kernel<4>, dim3(nblk(rows, 64)), dim3(256), 0, st, (const bf16*)x, (bf16*)y,
                         gamma, (long)rows, C, do_silu);
      SA_LAUNCH_CHECK();
      return SA_OK;
    }
    if (C == 192) {
      hipLaunchKernelGGL(rmsnorm_silu3_kernel<8>, dim3(nblk(rows, 32)), dim3(256), 0, st, (const bf16*)x, (bf16*)y,
                         gamma, (long)rows, C, do_silu);
      SA_LAUNCH_CHECK();
      return SA_OK;
    }
    if (C == 384) {
      hipLaunchKernelGGL(rmsnorm_silu3_kernel<16>, dim3(nblk(rows, 16)), dim3(256), 0, st, (const bf16*)x, (bf16*)y,
                         gamma, (long)rows, C, do_silu);
      SA_LAUNCH_CHECK();
      return SA_OK;
    }
  }
  if (g8 <= 16) {
    hipLaunchKernelGGL(rmsnorm_silu_kernel<16>, dim3(nblk(rows, 16)), dim3(256), 0, st, (const bf16*)x, (bf16*)y,
                       gamma, (long)rows, C, do_silu);
  } else if (g8 <= 32) {
    hipLaunchKernelGGL(rmsnorm_silu_kernel<32>, dim3(nblk(rows, 8)), dim3(256), 0, st, (const bf16*)x, (bf16*)y,
                       gamma, (long)rows, C, do_silu);
  } else {
    hipLaunchKernelGGL(rmsnorm_silu_kernel<64>, dim3(nblk(rows, 4)), dim3(256), 0, st, (const bf16*)x, (bf16*)y,
                       gamma, (long)rows, C, do_silu);
  }
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_vae_input(const float* z, int Cz, int64_t THW, const float* mean, const float* stdv, void* out,
                            int Cp, void* stream) {
  if (!z || !out || Cp < Cz) return SA_ERR_ARG;
  hipLaunchKernelGGL(vae_input_kernel, dim3(nblk(THW * Cp, 256)), dim3(256), 0, (hipStream_t)stream, z, Cz, THW,
                     mean, stdv, (bf16*)out, Cp);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_vae_output(const float* in, int C_stride, int C, int64_t THW, float* out, int post, void* stream) {
  if (!in || !out || C > C_stride) return SA_ERR_ARG;
  hipLaunchKernelGGL(vae_output_kernel, dim3(nblk(THW * C, 256)), dim3(256), 0, (hipStream_t)stream, in, C_stride, C,
                     THW, out, post);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_vae_latent_out(const float* in, int C_stride, int Cz, int64_t THW, const float* mean,
                                 const float* stdv, float* out, void* stream) {
  if (!in || !out || !mean || !stdv || 2 * Cz > C_stride) return SA_ERR_ARG;
  hipLaunchKernelGGL(vae_latent_out_kernel, dim3(nblk(THW * 2 * Cz, 256)), dim3(256), 0, (hipStream_t)stream, in,
                     C_stride, Cz, THW, mean, stdv, out);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_softmax_rows(const float* s, int64_t ld_s, void* p, int64_t ld_p, int64_t rows, int n, float scale,
                               void* stream) {
  if (!s || !p || rows <= 0 || n <= 0) return SA_ERR_ARG;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, s, ld_s, (bf16*)p,
                     ld_p, n, scale);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_transpose_bf16(const void* in, int64_t ld_in, int64_t stride_in, void* out, int64_t ld_out,
                                 int64_t stride_out, int rows, int cols, int batch, void* stream) {
  if (!in || !out) return SA_ERR_ARG;
  dim3 grid(nblk(cols, 32), nblk(rows, 32), batch);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16*)in, ld_in, stride_in,
                     (bf16*)out, ld_out, stride_out, rows, cols);
  SA_LAUNCH_CHECK();
  return SA_OK;
}
