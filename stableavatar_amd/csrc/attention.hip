// Flash-attention forward, bf16 in / fp32 softmax+accumulate / bf16 out, head_dim 128, no mask
// (the reference's SDPA path: wan_fantasy_transformer3d_1B.py:158-207 with q_lens/k_lens ignored,
// which it warns about at :190-193).  One kernel serves every attention site of the DiT:
//   * self-attention            (1B:402-407)   segments = batch rows, Lq = Lk = seq_len
//   * text / image cross-attn   (1B:556-570)   Lk = 512 / 257 (tail key block masked)
//   * per-frame vocal cross-attn(1B:575-586)   segments = (batch, latent frame), Lk = 17
// Segments come from a device table {q_row0, q_len, kv_row0, kv_len}; rows index flat
// [rows, stride] bf16 matrices with head h at column h*128, so Q/K/V are read straight out of
// the fused QKV GEMM output (no transposes).  ACCUMULATE adds into an existing bf16 output,
// which is how the three cross-attention terms are summed (1B:603).
//
// Structure (cdna_hip_programming.md App. B "Fused attention prefill"): 8 waves x 32 query rows,
// KV blocks of 64 keys staged by global_load_lds into a 2-deep LDS ring (XOR-swizzled 256-B rows).
// Swapped product S^T = K·Q^T puts one query per lane, so the online softmax is lane-local; P^T is
// fed back as the B operand straight from the accumulator and V^T comes from ds_read_b64_tr_b16,
// giving O^T with the query on the lane (rescale is per lane).  Self-attention runs the
// mfma_f32_16x16x32_bf16 block body (attn_v6_block), shared by the self-attention kernels and the fused
// cross-attention.
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace {

struct AttnArgs {
  const bf16* q; const bf16* k; const bf16* v; bf16* o;
  const int* segs;
  long qs, ks, vs, os;
  float c;  // softmax scale * log2(e)
  int accumulate;
  const int* orows;  // output row of query row r = orows[r] (null: r); the Ulysses exchange's receive layout
  // key-split launches (attn_fwd_v6_split_kernel): a 1-D grid whose first split_full workgroups are whole query tiles
  // and whose last 2 x split_n are the two key halves of the last split_n tiles (tile = (segment, head, query block),
  // nqb query blocks per segment, nheads heads); the halves write unnormalised fp32 partials to work
  int nqb, nheads, split_full, split_n;
  float* work;
};

constexpr int D = 128;
constexpr int WAVES = 8;
constexpr int QB = WAVES * 32;
constexpr int KVB = 64;
constexpr int TILE_BYTES = KVB * D * 2;      // 16 KB
constexpr int STAGE_BYTES = 2 * TILE_BYTES;  // K + V
constexpr int LDS_BYTES = 2 * STAGE_BYTES;   // 64 KB

// 16-byte chunk swizzle for 256-B rows: conflict-free for both row (ds_read_b128) and
// transposed (ds_read_b64_tr_b16) reads (cdna_hip_programming.md T10 form (b))
__device__ __forceinline__ int gsw(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

constexpr float RESCALE_THR = 8.0f;  // log2 units: P <= 2^8 between rescales (fused cross-attention)
// self-attention blocks (v6_softmax_p): the running max sits RESCALE_BIAS above the rows' maxima after each move, and
// the next move comes when a score passes its row's maximum by RESCALE_BIAS + 1 = RESCALE_THR
constexpr float RESCALE_BIAS = RESCALE_THR - 1.0f;

// non-canonicalising f32 max (MFMA outputs are never signalling NaNs): fmaxf makes hipcc insert a
// v_max_f32 x, x canonicalisation per operand (MI355X_MICROARCH.md, App. B attention pitfalls).  The
// IEEE-2019 maximum lowers to gfx950's v_maximum3_f32 with no canonicalisation, and, unlike an inline-asm
// v_max3_f32, needs no conservative s_nop after each link of a dependent chain (hipcc pads every VGPR an
// asm statement defines before the next VALU reads it: 16+ s_nop per block on the rescale test)
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}
__device__ __forceinline__ float vmax2(float a, float b) { return __builtin_elementwise_maximum(a, b); }
// LDS reads issued from inline asm at base+immediate addresses and retired by counted lgkmcnt waits
// (cdna_hip_programming.md §5.7 item 1 form (ii)), so hipcc neither serialises each fragment behind its own
// wait nor drains the next block's LDS-DMA (vmcnt(0)) before them
template <int OFF>
__device__ __forceinline__ void ds_b128(u32x4& d, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}
template <int OFF>
__device__ __forceinline__ void ds_tr64(u32x2& d, uint32_t addr) {
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}
template <int N>
__device__ __forceinline__ void wait_v(u32x2* f) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7])
               : "i"(N));
}
// The fused cross-attention keeps K and V of a block in separate 3-stage regions (K stage b at b * 16 KB,
// V stage b at 48 KB + b * 16 KB; the V read bases include the 48 KB) so a block's DMA is issued two blocks
// ahead
constexpr int X3_VBASE = 3 * TILE_BYTES, X3_LDS = 6 * TILE_BYTES;  // 96 KB

// ---- fused cross-attention of WanI2VTalkingCrossAttention (1B:556-603): per query block, the text
// (1B:564-570), image (1B:556-562) and per-frame vocal (1B:575-586) attentions run back to back over
// one K/V block stream, each with its own online softmax, and the three outputs are summed with the
// reference's bf16 rounding, (bf16(text) + bf16(img)) + bf16(vocal) (1B:602), so Q is read once and O
// written once.  A query block must lie inside one latent frame (tokens_per_frame % 256 == 0).
struct Cross3Args {
  const bf16* q; long qs;
  const bf16* kt; const bf16* vt; long ts; int t_len;
  const bf16* ki; const bf16* vi; long is; int i_len;
  const bf16* kv; const bf16* vv; long vs; int nper, tpf, n_frames, tok_offset;
  bf16* o; long os;
  int q_len;
  float c;
};

// ---- small-query attention for head dims the MFMA kernel does not take (vocal projector, D=192 for
// 1.3B and 640 for 14B, 17 queries per frame vs one latent frame's tokens: vocal_projector_fantasy_1B.py:
// 259-270, vocal_projector_fantasy_14B.py:254-267; wav2vec2, D=64).  One wave
// per (segment, head, query): scores for all keys in LDS, exact softmax, lane-parallel P·V.
constexpr int SMALL_MAXK = 4096;
constexpr int SMALL_MAXD = 640;

__global__ __launch_bounds__(256) void attn_small_kernel(const bf16* q, const bf16* k, const bf16* v, bf16* o,
                                                         const int* segs, int heads, int D, long qs, long ks, long vs,
                                                         long os, float scale) {
  __shared__ float p[4][SMALL_MAXK];
  __shared__ float qv[4][SMALL_MAXD];
  const int* sg = segs + blockIdx.z * 4;
  const int q_row0 = sg[0], q_len = sg[1], kv_row0 = sg[2], kv_len = sg[3];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qi = blockIdx.x * 4 + w;
  const int h = blockIdx.y;
  if (qi >= q_len) return;
  const bf16* qp = q + (long)(q_row0 + qi) * qs + h * D;
  for (int d = lane; d < D; d += 64) qv[w][d] = bf2f(qp[d]) * scale;
  __builtin_amdgcn_wave_barrier();
  float mx = -INFINITY;
  for (int j = lane; j < kv_len; j += 64) {
    const bf16* kp = k + (long)(kv_row0 + j) * ks + h * D;
    float s = 0.f;
    for (int d = 0; d < D; d += 8) {
      const bf16x8 kk = *(const bf16x8*)(kp + d);
#pragma unroll
      for (int t = 0; t < 8; ++t) s = fmaf(qv[w][d + t], bf2f(kk[t]), s);
    }
    p[w][j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < kv_len; j += 64) {
    const float e = __expf(p[w][j] - mx);
    p[w][j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __builtin_amdgcn_wave_barrier();
  const float inv = sum > 0.f ? 1.f / sum : 0.f;  // no keys: zeros, as SDPA
  bf16* op = o + (long)(q_row0 + qi) * os + h * D;
  for (int d = lane; d < D; d += 64) {
    float acc = 0.f;
    for (int j = 0; j < kv_len; ++j) acc = fmaf(p[w][j], bf2f(v[(long)(kv_row0 + j) * vs + h * D + d]), acc);
    op[d] = f2bf(acc * inv);
  }
}

// ---- small-query attention, head dim <= 256 (vocal projector D = 192, wav2vec2 D = 64, CLIP D = 80): one
// workgroup per (32-query chunk, head, segment), 4 waves x 8 queries; keys in chunks of 64 staged into LDS
// (K / V rows padded by 16 B: conflict-free row-per-lane b128 reads), scores with the key on the lane
// (Q broadcast from LDS, prescaled by scale·log2e), online softmax in fp32, then O with 4 head dims per
// lane.  The one-wave-per-query kernel above re-read K and V from L2 for every query (0.7 ms per vocal-
// projector call at config 2); this reads them once per 32 queries.
// Key split (nsplit > 1): the workgroups of a 32-query chunk each take kper keys and write their unnormalised O,
// running max and row sum to `work`, and attn_small2_combine_kernel merges them.  A sequence-parallel rank's vocal
// projector has 17 queries x 8 heads x 3 frames = 24 workgroups, each walking 1024 keys alone (0.28 ms per call at
// N = 8); split 8 ways, the same keys run on 192 CUs.
constexpr int SM2_D = 256, SM2_DP = SM2_D + 8, SM2_KC = 64, SM2_QW = 32;

// work block of one (segment, head, query chunk, split): O [32][D], then m [32], then l [32] (fp32)
__device__ __forceinline__ float* sm2_work_block(float* work, int seg, int h, int qc, int s, int heads, int nqc,
                                                 int nsplit, int D) {
  return work + ((((long)seg * heads + h) * nqc + qc) * nsplit + s) * (long)(SM2_QW * (D + 2));
}

__global__ __launch_bounds__(256) void attn_small2_kernel(const bf16* q, const bf16* k, const bf16* v, bf16* o,
                                                          const int* segs, int D, long qs, long ks, long vs, long os,
                                                          float c, int nsplit, int kper, float* work) {
  __shared__ __attribute__((aligned(16))) bf16 Ks[SM2_KC * SM2_DP];
  __shared__ __attribute__((aligned(16))) bf16 Vs[SM2_KC * SM2_DP];
  __shared__ __attribute__((aligned(16))) float Qs[SM2_QW * SM2_D];
  __shared__ __attribute__((aligned(16))) float Ps[4][8][SM2_KC];
  const int* sg = segs + blockIdx.z * 4;
  const int q_row0 = sg[0], q_len = sg[1], kv_row0 = sg[2], kv_len = sg[3];
  const int qc = blockIdx.x / nsplit, split = blockIdx.x % nsplit;
  const int q0 = qc * SM2_QW;
  if (q0 >= q_len) return;
  const int kb0 = split * kper, kb1 = min(kv_len, kb0 + kper);  // this workgroup's keys
  const int h = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int DP = D + 8, nch = D / 8;  // padded row (elements), 16-B chunks per row
  // Q rows of this chunk, fp32, prescaled (rows past q_len: zeros, never stored)
  for (int i = tid; i < SM2_QW * nch; i += 256) {
    const int r = i / nch, ch = i % nch;
    float* dst = Qs + r * SM2_D + ch * 8;
    if (q0 + r < q_len) {
      const bf16x8 x = *(const bf16x8*)(q + (long)(q_row0 + q0 + r) * qs + h * D + ch * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[j] = bf2f(x[j]) * c;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[j] = 0.f;
    }
  }
  float m[8], l[8], O[8][4];
#pragma unroll
  for (int qq = 0; qq < 8; ++qq) {
    m[qq] = -INFINITY;
    l[qq] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) O[qq][t] = 0.f;
  }
  const float* Qw = Qs + w * 8 * SM2_D;
  for (int kc = kb0; kc < kb1; kc += SM2_KC) {
    __syncthreads();  // previous chunk's K / V reads done (and Q written, first time)
    for (int i = tid; i < SM2_KC * nch; i += 256) {
      const int r = i / nch, ch = i % nch;
      u32x4 kx = {0u, 0u, 0u, 0u}, vx = {0u, 0u, 0u, 0u};
      if (kc + r < kb1) {
        kx = *(const u32x4*)(k + (long)(kv_row0 + kc + r) * ks + h * D + ch * 8);
        vx = *(const u32x4*)(v + (long)(kv_row0 + kc + r) * vs + h * D + ch * 8);
      }
      *(u32x4*)(Ks + r * DP + ch * 8) = kx;
      *(u32x4*)(Vs + r * DP + ch * 8) = vx;
    }
    __syncthreads();
    // scores of this lane's key for the wave's 8 queries
    float sc[8];
#pragma unroll
    for (int qq = 0; qq < 8; ++qq) sc[qq] = 0.f;
    for (int d = 0; d < D; d += 8) {
      const bf16x8 kk = *(const bf16x8*)(Ks + lane * DP + d);
      float kf[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[j] = bf2f(kk[j]);
#pragma unroll
      for (int qq = 0; qq < 8; ++qq) {
        const f32x4 a = *(const f32x4*)(Qw + qq * SM2_D + d), b = *(const f32x4*)(Qw + qq * SM2_D + d + 4);
        sc[qq] = fmaf(kf[0], a[0], sc[qq]); sc[qq] = fmaf(kf[1], a[1], sc[qq]);
        sc[qq] = fmaf(kf[2], a[2], sc[qq]); sc[qq] = fmaf(kf[3], a[3], sc[qq]);
        sc[qq] = fmaf(kf[4], b[0], sc[qq]); sc[qq] = fmaf(kf[5], b[1], sc[qq]);
        sc[qq] = fmaf(kf[6], b[2], sc[qq]); sc[qq] = fmaf(kf[7], b[3], sc[qq]);
      }
    }
    const bool valid = kc + lane < kb1;
#pragma unroll
    for (int qq = 0; qq < 8; ++qq) {
      const float s = valid ? sc[qq] : -INFINITY;
      const float m_new = fmaxf(m[qq], wave_max(s));  // finite: every chunk has a valid key
      const float alpha = __builtin_amdgcn_exp2f(m[qq] - m_new);
      const float p = __builtin_amdgcn_exp2f(s - m_new);
      l[qq] = l[qq] * alpha + wave_sum(p);
      m[qq] = m_new;
#pragma unroll
      for (int t = 0; t < 4; ++t) O[qq][t] *= alpha;
      Ps[w][qq][lane] = p;
    }
    __builtin_amdgcn_wave_barrier();  // the wave's own P writes before its broadcast reads (LDS is in order)
    // O[q][4 lane .. 4 lane + 3] += sum_j P[q][j] V[j][..]
    if (4 * lane < D) {
      for (int j = 0; j < SM2_KC; j += 4) {
        float vf[4][4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const bf16x4 vv = *(const bf16x4*)(Vs + (j + jj) * DP + 4 * lane);
#pragma unroll
          for (int t = 0; t < 4; ++t) vf[jj][t] = bf2f(vv[t]);
        }
#pragma unroll
        for (int qq = 0; qq < 8; ++qq) {
          const f32x4 p4 = *(const f32x4*)(&Ps[w][qq][j]);
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
#pragma unroll
            for (int t = 0; t < 4; ++t) O[qq][t] = fmaf(p4[jj], vf[jj][t], O[qq][t]);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // P reads done before the next chunk overwrites P
  }
  if (nsplit > 1) {  // partial result (a split with no keys: m = -inf, l = 0, O = 0)
    float* blk = sm2_work_block(work, blockIdx.z, h, qc, split, gridDim.y, (gridDim.x + nsplit - 1) / nsplit,
                                nsplit, D);
#pragma unroll
    for (int qq = 0; qq < 8; ++qq) {
      const int r = w * 8 + qq;
      if (q0 + r < q_len) {
        if (4 * lane < D) *(f32x4*)(blk + r * D + 4 * lane) = (f32x4){O[qq][0], O[qq][1], O[qq][2], O[qq][3]};
        if (lane == 0) {
          blk[SM2_QW * D + r] = m[qq];
          blk[SM2_QW * D + SM2_QW + r] = l[qq];
        }
      }
    }
    return;
  }
  if (4 * lane < D) {
#pragma unroll
    for (int qq = 0; qq < 8; ++qq) {
      const int qi = q0 + w * 8 + qq;
      if (qi < q_len) {
        const float inv = l[qq] > 0.f ? 1.f / l[qq] : 0.f;  // a segment with no keys: zeros, as SDPA
        *(bf16x4*)(o + (long)(q_row0 + qi) * os + h * D + 4 * lane) =
            (bf16x4){f2bf(O[qq][0] * inv), f2bf(O[qq][1] * inv), f2bf(O[qq][2] * inv), f2bf(O[qq][3] * inv)};
      }
    }
  }
}

// merge of the key splits: O = sum_s 2^(m_s - M) O_s / sum_s 2^(m_s - M) l_s, M = max_s m_s (m in log2 units)
__global__ __launch_bounds__(256) void attn_small2_combine_kernel(bf16* o, const int* segs, int D, long os,
                                                                  int nsplit, const float* work) {
  const int* sg = segs + blockIdx.z * 4;
  const int q_row0 = sg[0], q_len = sg[1];
  const int qc = blockIdx.x, q0 = qc * SM2_QW, h = blockIdx.y;
  if (q0 >= q_len) return;
  const int nq = min(SM2_QW, q_len - q0), n4 = D / 4;
  const float* blk0 = sm2_work_block(const_cast<float*>(work), blockIdx.z, h, qc, 0, gridDim.y, gridDim.x, nsplit, D);
  const long bstride = (long)SM2_QW * (D + 2);
  for (int i = threadIdx.x; i < nq * n4; i += 256) {
    const int r = i / n4, d = (i % n4) * 4;
    float M = -INFINITY;
    for (int s = 0; s < nsplit; ++s) M = fmaxf(M, blk0[s * bstride + SM2_QW * D + r]);
    float L = 0.f;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (M != -INFINITY) {
      for (int s = 0; s < nsplit; ++s) {
        const float* b = blk0 + s * bstride;
        const float a = __builtin_amdgcn_exp2f(b[SM2_QW * D + r] - M);
        L += a * b[SM2_QW * D + SM2_QW + r];
        const f32x4 x = *(const f32x4*)(b + r * D + d);
        acc[0] += a * x[0]; acc[1] += a * x[1]; acc[2] += a * x[2]; acc[3] += a * x[3];
      }
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;  // no keys at all: zeros, as SDPA
    *(bf16x4*)(o + (long)(q_row0 + q0 + r) * os + h * D + d) =
        (bf16x4){f2bf(acc[0] * inv), f2bf(acc[1] * inv), f2bf(acc[2] * inv), f2bf(acc[3] * inv)};
  }
}

}  // namespace

static bool sm2_applies(const void* q, const void* v, const void* o, int head_dim, int64_t q_stride, int64_t v_stride,
                        int64_t o_stride) {
  return head_dim <= SM2_D && !(q_stride % 8) && !(v_stride % 8) && !(o_stride % 4) &&
         !(((uintptr_t)q | (uintptr_t)v) & 15) && !(((uintptr_t)o) & 7);
}

extern "C" int sa_attn_small(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg,
                             int max_q_len, int max_kv_len, int heads, int head_dim, int64_t q_stride,
                             int64_t k_stride, int64_t v_stride, int64_t o_stride, float scale, void* stream);

extern "C" int sa_attn_small_split(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg,
                                   int max_q_len, int max_kv_len, int heads, int head_dim, int64_t q_stride,
                                   int64_t k_stride, int64_t v_stride, int64_t o_stride, float scale, int nsplit,
                                   void* work, int64_t work_bytes, void* stream) {
  if (!q || !k || !v || !o || !segs || nseg <= 0 || max_q_len <= 0 || heads <= 0 || nsplit < 2) return SA_ERR_ARG;
  if (head_dim <= 0 || head_dim % 8 || max_kv_len <= 0 || (k_stride % 8) || (((uintptr_t)k) & 15)) return SA_ERR_ARG;
  if (!sm2_applies(q, v, o, head_dim, q_stride, v_stride, o_stride)) return SA_ERR_ARG;
  const int nchunks = (max_kv_len + SM2_KC - 1) / SM2_KC;
  const int per = (nchunks + nsplit - 1) / nsplit;  // 64-key chunks per split
  nsplit = (nchunks + per - 1) / per;               // no split without keys at the longest segment
  const int nqc = (max_q_len + SM2_QW - 1) / SM2_QW;
  const int64_t need = (int64_t)nseg * heads * nqc * nsplit * SM2_QW * (head_dim + 2) * 4;
  if (!work || (((uintptr_t)work) & 15) || work_bytes < need) return SA_ERR_ARG;
  if (nsplit < 2) return sa_attn_small(q, k, v, o, segs, nseg, max_q_len, max_kv_len, heads, head_dim, q_stride,
                                       k_stride, v_stride, o_stride, scale, stream);
  hipLaunchKernelGGL(attn_small2_kernel, dim3(nqc * nsplit, heads, nseg), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, segs, head_dim, q_stride, k_stride,
                     v_stride, o_stride, scale * 1.4426950408889634f, nsplit, per * SM2_KC, (float*)work);
  SA_LAUNCH_CHECK();
  hipLaunchKernelGGL(attn_small2_combine_kernel, dim3(nqc, heads, nseg), dim3(256), 0, (hipStream_t)stream, (bf16*)o,
                     segs, head_dim, o_stride, nsplit, (const float*)work);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_attn_small(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg,
                             int max_q_len, int max_kv_len, int heads, int head_dim, int64_t q_stride,
                             int64_t k_stride, int64_t v_stride, int64_t o_stride, float scale, void* stream) {
  if (!q || !k || !v || !o || !segs || nseg <= 0 || max_q_len <= 0 || heads <= 0) return SA_ERR_ARG;
  if (head_dim <= 0 || head_dim > SMALL_MAXD || head_dim % 8 || max_kv_len <= 0) return SA_ERR_ARG;
  if ((k_stride % 8) || (((uintptr_t)k) & 15)) return SA_ERR_ARG;
  // the tiled kernel: 16-byte Q / K / V row chunks, 8-byte O stores (head_dim % 8 == 0 already holds)
  if (sm2_applies(q, v, o, head_dim, q_stride, v_stride, o_stride)) {
    dim3 grid2((max_q_len + SM2_QW - 1) / SM2_QW, heads, nseg);
    hipLaunchKernelGGL(attn_small2_kernel, grid2, dim3(256), 0, (hipStream_t)stream, (const bf16*)q, (const bf16*)k,
                       (const bf16*)v, (bf16*)o, segs, head_dim, q_stride, k_stride, v_stride, o_stride,
                       scale * 1.4426950408889634f, 1, max_kv_len, (float*)nullptr);
    SA_LAUNCH_CHECK();
    return SA_OK;
  }
  if (max_kv_len > SMALL_MAXK) return SA_ERR_ARG;  // the one-wave-per-query kernel keeps a score row in LDS
  dim3 grid((max_q_len + 3) / 4, heads, nseg);
  hipLaunchKernelGGL(attn_small_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16*)q, (const bf16*)k,
                     (const bf16*)v, (bf16*)o, segs, heads, head_dim, q_stride, k_stride, v_stride, o_stride, scale);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

// ---- v6: v3's pipeline (2-deep K/V ring by LDS-DMA, asm LDS reads with counted waits, prescaled Q
// and -m as the QK^T initial accumulator, deferred rescale) on mfma_f32_16x16x32_bf16 instead of
// 32x32x16.  The two shapes take the same cycles per FLOP, but under load the chip holds a higher
// clock on the 16x16x32 stream (MI355X_MICROARCH.md "DVFS give-back" item 7: ~1.12-1.15x FLOP/s on
// random data).  Per wave: 32 queries as two 16-query tiles, 64-key blocks as four 16-key tiles.
//   S^T tile (kt, qt) = K_kt · Q_qt^T: lane holds keys 4g+i (g = lane/16) of tile kt for query lane%16
//   P^T as the PV B operand: the 32-key chunk c is taken in the permuted key order
//     k = 8g + j -> key 32c + 4g + j (j < 4), 32c + 16 + 4g + j - 4 (j >= 4)
//   so a lane's 8 P values are its own S^T registers of tiles 2c and 2c+1 (no lane exchange), and the
//   V^T A operand uses the same order: two ds_read_b64_tr_b16 (rows 32c+4g.. and 32c+16+4g..)
//   row max over 64 keys: 15 VALU max + permlane32 / permlane16 swaps; row sums stay per lane until
//   the end.
// LDS images: K rows chunk ^ (row & 15) (conflict-free 16-row b128 reads), V rows chunk ^ 2(row & 7)
// (conflict-free transposed reads).
__device__ __forceinline__ bf16x8 v6_as_bf8(u32x4 x) { return __builtin_bit_cast(bf16x8, x); }
__device__ __forceinline__ bf16x8 v6_as_bf8(u32x2 lo, u32x2 hi) {
  const u32x4 x = {lo[0], lo[1], hi[0], hi[1]};
  return __builtin_bit_cast(bf16x8, x);
}

// K fragments of key tile KT (d chunks 0-3) of the K stage at byte KOFF from the K read bases
template <int KOFF, int KT>
__device__ __forceinline__ void v6_read_k(u32x4* f, const uint32_t* ka) {
  constexpr int base = KOFF + KT * 4096;
  ds_b128<base>(f[0], ka[0]);
  ds_b128<base>(f[1], ka[1]);
  ds_b128<base>(f[2], ka[2]);
  ds_b128<base>(f[3], ka[3]);
}
// V^T fragments of key chunk C for d tiles DT0..DT0+3 of the V stage at byte VOFF from the V read bases:
// f[2*t + h], h = rows +0 / +16
template <int VOFF, int C, int DT0>
__device__ __forceinline__ void v6_read_v(u32x2* f, const uint32_t* va) {
  constexpr int base = VOFF + C * 8192;
  ds_tr64<base>(f[0], va[DT0 + 0]); ds_tr64<base + 4096>(f[1], va[DT0 + 0]);
  ds_tr64<base>(f[2], va[DT0 + 1]); ds_tr64<base + 4096>(f[3], va[DT0 + 1]);
  ds_tr64<base>(f[4], va[DT0 + 2]); ds_tr64<base + 4096>(f[5], va[DT0 + 2]);
  ds_tr64<base>(f[6], va[DT0 + 3]); ds_tr64<base + 4096>(f[7], va[DT0 + 3]);
}
__device__ __forceinline__ void v6_mma_k(f32x4 (&S)[4][2], int kt, const u32x4* f, const bf16x8 (&qf)[2][4]) {
#pragma unroll
  for (int dc = 0; dc < 4; ++dc) {
    S[kt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v6_as_bf8(f[dc]), qf[0][dc], S[kt][0], 0, 0, 0);
    S[kt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v6_as_bf8(f[dc]), qf[1][dc], S[kt][1], 0, 0, 0);
  }
}
__device__ __forceinline__ void v6_mma_v(f32x4 (&O)[8][2], int dt0, const u32x2* f, const bf16x8 (&pb)[2]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bf16x8 a = v6_as_bf8(f[2 * t], f[2 * t + 1]);
    O[dt0 + t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb[0], O[dt0 + t][0], 0, 0, 0);
    O[dt0 + t][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb[1], O[dt0 + t][1], 0, 0, 0);
  }
}
template <int N>
__device__ __forceinline__ void wait_k4(u32x4* f) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]) : "i"(N));
}

struct V6State {
  f32x4 O[8][2];
  f32x4 L[2];     // row sums of the bf16 P (every element equal), from a ones x P^T MFMA
  float negm[2];  // -m per query tile (this lane's query)
  f32x4 negm4[2];  // the same as the QK^T chains' initial accumulator (refreshed only on a rescale)
};

// max over 16 values of one query's S^T column slice, then over the 4 lane groups (permlane32 / 16 swaps)
__device__ __forceinline__ float rowmax64(const f32x4 (&S)[4][2], int qt) {
  float m = vmax3(S[0][qt][0], S[0][qt][1], S[0][qt][2]);
  m = vmax3(m, S[0][qt][3], S[1][qt][0]);
  m = vmax3(m, S[1][qt][1], S[1][qt][2]);
  m = vmax3(m, S[1][qt][3], S[2][qt][0]);
  m = vmax3(m, S[2][qt][1], S[2][qt][2]);
  m = vmax3(m, S[2][qt][3], S[3][qt][0]);
  m = vmax3(m, S[3][qt][1], S[3][qt][2]);
  m = vmax2(m, S[3][qt][3]);
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  m = vmax2(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return vmax2(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// max over this lane's 32 scores (both query tiles), as a 3-ary tree (depth 4 instead of a 16-long chain)
__device__ __forceinline__ float lanemax32(const f32x4 (&S)[4][2]) {
  float v[32];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int i = 0; i < 4; ++i) v[kt * 8 + qt * 4 + i] = S[kt][qt][i];
  float r[12];
#pragma unroll
  for (int j = 0; j < 10; ++j) r[j] = vmax3(v[3 * j], v[3 * j + 1], v[3 * j + 2]);
  r[10] = v[30];
  r[11] = v[31];
  const float a = vmax3(r[0], r[1], r[2]), b = vmax3(r[3], r[4], r[5]), c = vmax3(r[6], r[7], r[8]),
              d = vmax3(r[9], r[10], r[11]);
  return vmax2(vmax3(a, b, c), d);
}

// the fused cross-attention's softmax step (attn_v6_block<.., false>): the rescale test on the scores (a lane max
// over its 32 scores against RESCALE_THR, no row reduction unless it fails), the exponentials in place in S.  It
// keeps the cross-attention kernels inside 256 VGPRs with the fewest spills (the P-side test of v6_softmax_p holds
// the scores and the packed P of the whole block at once)
__device__ __forceinline__ void v6_softmax_s(V6State& st, f32x4 (&S)[4][2], const bool FIRST) {
  if (FIRST || !__all(lanemax32(S) <= RESCALE_THR)) {  // wave-uniform
    float mx[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) mx[qt] = rowmax64(S, qt);  // max of c S - m over the block's 64 keys
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float delta = FIRST ? mx[qt] : fmaxf(mx[qt], 0.f);
      if (!FIRST) {  // O and L are still zero on the first block (no 0 x inf for a very negative max)
        const float alpha = __builtin_amdgcn_exp2f(-delta);
        st.L[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
#pragma unroll
          for (int i = 0; i < 4; ++i) st.O[dt][qt][i] *= alpha;
      }
      st.negm[qt] -= delta;
      st.negm4[qt] = (f32x4){st.negm[qt], st.negm[qt], st.negm[qt], st.negm[qt]};
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) S[kt][qt][i] -= delta;
    }
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) S[kt][qt][i] = __builtin_amdgcn_exp2f(S[kt][qt][i]);
}

// P = bf16(exp2(S)) of a block in PV operand order (pb[c][qt]: key tiles 2c, 2c+1 of query tile qt); S is kept
__device__ __forceinline__ void v6_pack_exp(const f32x4 (&S)[4][2], bf16x8 (&pb)[2][2]) {
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pb[c][qt][j] = f2bf(__builtin_amdgcn_exp2f(S[2 * c][qt][j]));
        pb[c][qt][4 + j] = f2bf(__builtin_amdgcn_exp2f(S[2 * c + 1][qt][j]));
      }
}

// The online-softmax step of one 64-key block (attn_v6_block, attn_v6t_block): P into pb, the running max moved
// first where needed.  The running max is kept RESCALE_BIAS log2 units above the rows' maxima (P <= 2^-7 right after
// a move), and the test runs on the bf16 P: some P >= 2 -- a score 8 above its row's maximum -- iff bit 14 of some
// packed P is set (P >= 0: biased exponent >= 128), so the OR of the 16 P dwords (8 v_or3) decides, where a max tree
// over the 32 scores took 16 ops (6.08-6.18 vs 6.19-6.22 ms per config-2 launch).  The first block, or a failed test,
// moves the running max of every row whose block maximum passes it, rescales O and L and forms P again from S.
template <bool FIRST_CT>
__device__ __forceinline__ void v6_softmax_p(V6State& st, f32x4 (&S)[4][2], bf16x8 (&pb)[2][2], bool first_rt) {
  const bool FIRST = FIRST_CT || first_rt;
  bool move = FIRST;
  if (!FIRST) {
    v6_pack_exp(S, pb);
    u32x4 w[4];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) w[2 * c + qt] = __builtin_bit_cast(u32x4, pb[c][qt]);
    // a depth-3 tree of v_or3 (a 7-long dependent chain measured 0.5 % slower, attn_or_tree_ab_r6tr.jsonl)
    const uint32_t a = w[0][0] | w[0][1] | w[0][2], b = w[0][3] | w[1][0] | w[1][1], c = w[1][2] | w[1][3] | w[2][0],
                   d = w[2][1] | w[2][2] | w[2][3], e = w[3][0] | w[3][1] | w[3][2];
    const uint32_t acc = (a | b | c) | (d | e | w[3][3]);
    move = !__all((acc & 0x40004000u) == 0u);  // wave-uniform
  }
  if (move) {
    float mx[2], alpha[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) mx[qt] = rowmax64(S, qt);  // max of c S - m over the block's 64 keys
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float delta = FIRST ? mx[qt] + RESCALE_BIAS : fmaxf(mx[qt] + RESCALE_BIAS, 0.f);
      alpha[qt] = __builtin_amdgcn_exp2f(-delta);
      st.negm[qt] -= delta;
      st.negm4[qt] = (f32x4){st.negm[qt], st.negm[qt], st.negm[qt], st.negm[qt]};
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) S[kt][qt][i] -= delta;
    }
    if (!FIRST)  // O and L are still zero on the first block (no 0 x inf for a very negative max)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        st.L[qt] *= alpha[qt];
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
#pragma unroll
          for (int i = 0; i < 4; ++i) st.O[dt][qt][i] *= alpha[qt];
      }
    v6_pack_exp(S, pb);
  }
}

// one 64-key block whose K / V stages sit at KOFF / VOFF from the read bases (self-attention: K and V of a
// stage adjacent in a 2-stage ring; the fused cross-attention: separate 3-stage K and V regions).  The first
// block of a softmax sets the running max: FIRST_CT at compile time (self-attention), first_rt per source
// (cross-attention)
template <int KOFF, int VOFF, bool FIRST_CT, bool PTEST = true>
__device__ __forceinline__ void attn_v6_block(V6State& st, const bf16x8 (&qf)[2][4], const uint32_t* ka,
                                              const uint32_t* va, int kb, int kv_len, int g,
                                              bool first_rt = false) {
  f32x4 S[4][2];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
      S[kt][qt] = st.negm4[qt];
  // S'^T = c K Q^T - m, K fragments two key tiles ahead
  u32x4 k0[4], k1[4];
  v6_read_k<KOFF, 0>(k0, ka);
  v6_read_k<KOFF, 1>(k1, ka);
  wait_k4<4>(k0);
  v6_mma_k(S, 0, k0, qf);
  v6_read_k<KOFF, 2>(k0, ka);
  wait_k4<4>(k1);
  v6_mma_k(S, 1, k1, qf);
  v6_read_k<KOFF, 3>(k1, ka);
  wait_k4<4>(k0);
  v6_mma_k(S, 2, k0, qf);
  wait_k4<0>(k1);
  v6_mma_k(S, 3, k1, qf);
  // first V^T fragments under the softmax
  u32x2 v0[8], v1[8];
  v6_read_v<VOFF, 0, 0>(v0, va);
  v6_read_v<VOFF, 0, 4>(v1, va);

  if (kb * KVB + KVB > kv_len) {
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (kb * KVB + kt * 16 + 4 * g + i >= kv_len) { S[kt][0][i] = -INFINITY; S[kt][1][i] = -INFINITY; }
  }
  // PTEST: the self-attention kernels' step (P-side rescale test, P for the whole block); else the fused
  // cross-attention's (v6_softmax_s: P formed per key chunk below)
  bf16x8 pb[2][2];
  if constexpr (PTEST) v6_softmax_p<FIRST_CT>(st, S, pb, first_rt);
  else v6_softmax_s(st, S, FIRST_CT || first_rt);
  // O^T += V^T P^T, key chunk c = tiles (2c, 2c+1)
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if constexpr (!PTEST)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pb[c][qt][j] = f2bf(S[2 * c][qt][j]);
          pb[c][qt][4 + j] = f2bf(S[2 * c + 1][qt][j]);
        }
    {
      bf16x8 ones;
#pragma unroll
      for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;
      st.L[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[c][0], st.L[0], 0, 0, 0);
      st.L[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[c][1], st.L[1], 0, 0, 0);
    }
    if (c == 0) {
      wait_v<8>(v0);
      v6_mma_v(st.O, 0, v0, pb[c]);
      v6_read_v<VOFF, 1, 0>(v0, va);
      wait_v<8>(v1);
      v6_mma_v(st.O, 4, v1, pb[c]);
      v6_read_v<VOFF, 1, 4>(v1, va);
    } else {
      wait_v<8>(v0);
      v6_mma_v(st.O, 0, v0, pb[c]);
      wait_v<0>(v1);
      v6_mma_v(st.O, 4, v1, pb[c]);
    }
  }
}

// ---- V^T forms of the block (V read as V^T from a d-major producer layout, [H*128][Rv] bf16: row h*128 + d holds
// d of head h for every key row), so each PV operand is ds_read_b128 instead of two ds_read_b64_tr_b16.
// v6t: the v6 block with V^T staged 128 d-rows x 64 keys (128 B per d-row, 16-B chunk c of row d at position
//   c ^ (d & 7)); the producer stores the keys of each 32-key chunk in P's permuted order (position 8g + j <-> key
//   4g + j, j < 4; 16 + 4g + j - 4, j >= 4), so a lane's 16x16x32 PV operand is one b128 read.  (Measured and
//   removed, records under profiles/r05/: the PV product on 32x32x16 MFMAs, a two-wave ping-pong, a 3-stage ring.)
template <int VOFF, int C, int T0>
__device__ __forceinline__ void v6t_read_v(u32x4* f, const uint32_t* vb) {
  ds_b128<VOFF + (T0 + 0) * 2048>(f[0], vb[C]);
  ds_b128<VOFF + (T0 + 1) * 2048>(f[1], vb[C]);
  ds_b128<VOFF + (T0 + 2) * 2048>(f[2], vb[C]);
  ds_b128<VOFF + (T0 + 3) * 2048>(f[3], vb[C]);
}
__device__ __forceinline__ void v6t_mma_v(f32x4 (&O)[8][2], int dt0, const u32x4* f, const bf16x8 (&pb)[2]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bf16x8 a = v6_as_bf8(f[t]);
    O[dt0 + t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb[0], O[dt0 + t][0], 0, 0, 0);
    O[dt0 + t][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb[1], O[dt0 + t][1], 0, 0, 0);
  }
}

template <int KOFF>
__device__ __forceinline__ void v6_qk(f32x4 (&S)[4][2], const f32x4 (&negm4)[2], const bf16x8 (&qf)[2][4],
                                      const uint32_t* ka) {
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) S[kt][qt] = negm4[qt];
  u32x4 k0[4], k1[4];
  v6_read_k<KOFF, 0>(k0, ka);
  v6_read_k<KOFF, 1>(k1, ka);
  wait_k4<4>(k0);
  v6_mma_k(S, 0, k0, qf);
  v6_read_k<KOFF, 2>(k0, ka);
  wait_k4<4>(k1);
  v6_mma_k(S, 1, k1, qf);
  v6_read_k<KOFF, 3>(k1, ka);
  wait_k4<4>(k0);
  v6_mma_k(S, 2, k0, qf);
  wait_k4<0>(k1);
  v6_mma_k(S, 3, k1, qf);
}

__device__ __forceinline__ void v6_tail_mask(f32x4 (&S)[4][2], int kb, int kv_len, int g) {
  if (kb * KVB + KVB > kv_len) {
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (kb * KVB + kt * 16 + 4 * g + i >= kv_len) { S[kt][0][i] = -INFINITY; S[kt][1][i] = -INFINITY; }
  }
}

template <int KOFF, int VOFF, bool FIRST>
__device__ __forceinline__ void attn_v6t_block(V6State& st, const bf16x8 (&qf)[2][4], const uint32_t* ka,
                                               const uint32_t* vb, int kb, int kv_len, int g) {
  f32x4 S[4][2];
  v6_qk<KOFF>(S, st.negm4, qf, ka);
  u32x4 v0[4], v1[4];
  v6t_read_v<VOFF, 0, 0>(v0, vb);
  v6t_read_v<VOFF, 0, 4>(v1, vb);
  v6_tail_mask(S, kb, kv_len, g);
  bf16x8 pb[2][2];
  v6_softmax_p<FIRST>(st, S, pb, false);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    {
      bf16x8 ones;
#pragma unroll
      for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;
      st.L[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[c][0], st.L[0], 0, 0, 0);
      st.L[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[c][1], st.L[1], 0, 0, 0);
    }
    if (c == 0) {
      wait_k4<4>(v0);
      v6t_mma_v(st.O, 0, v0, pb[c]);
      v6t_read_v<VOFF, 1, 0>(v0, vb);
      wait_k4<4>(v1);
      v6t_mma_v(st.O, 4, v1, pb[c]);
      v6t_read_v<VOFF, 1, 4>(v1, vb);
    } else {
      wait_k4<4>(v0);
      v6t_mma_v(st.O, 0, v0, pb[c]);
      wait_k4<0>(v1);
      v6t_mma_v(st.O, 4, v1, pb[c]);
    }
  }
}

// the fused cross-attention's last block of a source with at most 32 keys left (the image's 257th key, the 32
// vocal keys of a frame): attn_v6_block on key tiles 0-1 only -- half the QK^T / PV MFMAs and exponentials
__device__ __forceinline__ float rowmax32_c0(const f32x4 (&S)[2][2], int qt) {
  float m = vmax3(S[0][qt][0], S[0][qt][1], S[0][qt][2]);
  m = vmax3(m, S[0][qt][3], S[1][qt][0]);
  m = vmax3(m, S[1][qt][1], S[1][qt][2]);
  m = vmax2(m, S[1][qt][3]);
  const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  m = vmax2(__uint_as_float(x[0]), __uint_as_float(x[1]));
  const auto y = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return vmax2(__uint_as_float(y[0]), __uint_as_float(y[1]));
}

template <int KOFF, int VOFF>
__device__ __forceinline__ void attn_half_block(V6State& st, const bf16x8 (&qf)[2][4], const uint32_t* ka,
                                                const uint32_t* va, int kb, int kv_len, int g, bool first) {
  f32x4 S[2][2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) S[kt][qt] = st.negm4[qt];
  u32x4 k0[4], k1[4];
  v6_read_k<KOFF, 0>(k0, ka);
  v6_read_k<KOFF, 1>(k1, ka);
  wait_k4<4>(k0);
#pragma unroll
  for (int dc = 0; dc < 4; ++dc) {
    S[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v6_as_bf8(k0[dc]), qf[0][dc], S[0][0], 0, 0, 0);
    S[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v6_as_bf8(k0[dc]), qf[1][dc], S[0][1], 0, 0, 0);
  }
  wait_k4<0>(k1);
#pragma unroll
  for (int dc = 0; dc < 4; ++dc) {
    S[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v6_as_bf8(k1[dc]), qf[0][dc], S[1][0], 0, 0, 0);
    S[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v6_as_bf8(k1[dc]), qf[1][dc], S[1][1], 0, 0, 0);
  }
  u32x2 v0[8], v1[8];
  v6_read_v<VOFF, 0, 0>(v0, va);
  v6_read_v<VOFF, 0, 4>(v1, va);
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (kb * KVB + kt * 16 + 4 * g + i >= kv_len) { S[kt][0][i] = -INFINITY; S[kt][1][i] = -INFINITY; }
  float lm = vmax3(S[0][0][0], S[0][0][1], S[0][0][2]);
  lm = vmax3(lm, S[0][0][3], S[0][1][0]);
  lm = vmax3(lm, S[0][1][1], S[0][1][2]);
  lm = vmax3(lm, S[0][1][3], S[1][0][0]);
  lm = vmax3(lm, S[1][0][1], S[1][0][2]);
  lm = vmax3(lm, S[1][0][3], S[1][1][0]);
  lm = vmax3(lm, S[1][1][1], S[1][1][2]);
  lm = vmax2(lm, S[1][1][3]);
  if (first || !__all(lm <= RESCALE_THR)) {  // wave-uniform
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float mx = rowmax32_c0(S, qt);
      const float delta = first ? mx : fmaxf(mx, 0.f);
      if (!first) {
        const float alpha = __builtin_amdgcn_exp2f(-delta);
        st.L[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
#pragma unroll
          for (int i = 0; i < 4; ++i) st.O[dt][qt][i] *= alpha;
      }
      st.negm[qt] -= delta;
      st.negm4[qt] = (f32x4){st.negm[qt], st.negm[qt], st.negm[qt], st.negm[qt]};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) S[kt][qt][i] -= delta;
    }
  }
  bf16x8 pb[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pb[qt][j] = f2bf(__builtin_amdgcn_exp2f(S[0][qt][j]));
      pb[qt][4 + j] = f2bf(__builtin_amdgcn_exp2f(S[1][qt][j]));
    }
  {
    bf16x8 ones;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;
    st.L[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[0], st.L[0], 0, 0, 0);
    st.L[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[1], st.L[1], 0, 0, 0);
  }
  wait_v<8>(v0);
  v6_mma_v(st.O, 0, v0, pb);
  wait_v<0>(v1);
  v6_mma_v(st.O, 4, v1, pb);
}

namespace {

// NW = 8: 256 query rows per workgroup, waves w and w+4 share a SIMD (one workgroup per CU); NW = 4: 128
// query rows, one wave per SIMD, two workgroups per CU -- the same per-SIMD pairing at half the work
// granularity, for launches whose 256-row workgroup count leaves the last round over the CUs mostly empty
// (the per-rank shapes of Ulysses SP: 378 workgroups at N = 8)
// SPLIT: the key-split launch (AttnArgs split_*): a half workgroup runs the flash loop over its half of the keys and
// writes O (unnormalised), the running max and the row sum instead of the output; attn_split_merge_kernel combines the
// two halves
template <int NW, bool SPLIT = false>
__device__ __forceinline__ void attn_fwd_v6_body(const AttnArgs& a) {
  constexpr int QBW = NW * 32, PPW = 16 / NW;  // query rows per workgroup, K (and V) 1-KB pieces per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int qb, h, seg, half = -1, stile = 0;
  if constexpr (SPLIT) {
    int tile;
    if ((int)blockIdx.x < a.split_full) {
      tile = xcd_remap(blockIdx.x, a.split_full);
    } else {
      const int idx = blockIdx.x - a.split_full;
      stile = idx >> 1;
      half = idx & 1;
      tile = a.split_full + stile;
    }
    qb = tile % a.nqb;
    h = (tile / a.nqb) % a.nheads;
    seg = tile / (a.nqb * a.nheads);
  } else {
    const int nx = gridDim.x, ny = gridDim.y;
    const int flat = xcd_remap(blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z), nx * ny * gridDim.z);
    qb = flat % nx;
    h = (flat / nx) % ny;
    seg = flat / (nx * ny);
  }
  const int* sg = a.segs + seg * 4;
  const int q_row0 = sg[0], q_len = sg[1];
  int kv_row0 = sg[2], kv_len = sg[3];
  if (SPLIT && half >= 0) {  // this half's keys: whole 64-key blocks in the first half
    const int kper = ((kv_len + 1) / 2 + KVB - 1) / KVB * KVB;
    if (half == 0) {
      kv_len = min(kv_len, kper);
    } else {
      kv_row0 += kper;
      kv_len -= kper;
    }
  }
  if (qb * QBW >= q_len) return;
  const int tid = threadIdx.x, lane = tid & 63;
  float* const wblk = SPLIT && half >= 0 ? a.work + ((long)stile * 2 + half) * QBW * (D + 2) : nullptr;
  if (SPLIT && half >= 0 && kv_len <= 0) {  // an empty half: m = -inf, l = 0, O = 0
    for (int i = tid; i < QBW * D; i += NW * 64) wblk[i] = 0.f;
    for (int i = tid; i < QBW; i += NW * 64) {
      wblk[QBW * D + i] = -INFINITY;
      wblk[QBW * D + QBW + i] = 0.f;
    }
    return;
  }
  if (kv_len <= 0) {  // a segment with no keys: zeros, as SDPA (nothing to add when accumulating)
    if (!a.accumulate)
      for (int i = tid; i < QBW * (D / 8); i += NW * 64) {
        const int qi = qb * QBW + i / (D / 8);
        if (qi < q_len) {
          const int orow = a.orows ? a.orows[q_row0 + qi] : q_row0 + qi;
          *(u32x4*)(a.o + (long)orow * a.os + h * D + (i % (D / 8)) * 8) = (u32x4){0u, 0u, 0u, 0u};
        }
      }
    return;
  }
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;

  // Q as the B operand: query tile qt, d chunk dc: Q[query][dc*32 + 8g .. +7], prescaled by c
  bf16x8 qf[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qc = min(qb * QBW + wave * 32 + qt * 16 + r16, q_len - 1);
    const bf16* qp = a.q + (long)(q_row0 + qc) * a.qs + h * D + 8 * g;
#pragma unroll
    for (int dc = 0; dc < 4; ++dc) {
      qf[qt][dc] = *(const bf16x8*)(qp + 32 * dc);
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[qt][dc][j] = f2bf(bf2f(qf[qt][dc][j]) * a.c);
    }
  }

  // K/V pieces: each wave moves 2 x 1-KB pieces (4 rows each) of K and of V per block; lane -> row
  // (lane / 16), stored position lane % 16 holding source chunk (lane % 16) ^ swizzle(row).  By
  // buffer_load...lds from SGPR descriptors, per-lane 32-bit offsets and the block in soffset: no 64-bit
  // address VALU.  The range check takes voffset + soffset + the instruction offset against the records (a V^T
  // form reading per-source chunks, measured and removed in round 6, read zeros past a records value that left
  // soffset out); a partial last block is staged from a descriptor of its own (base = its first row, soffset 0)
  // whose range ends at the segment's last row, so its rows past kv_len read as zeros (masked in S, and 0 x 0 in
  // PV) instead of whatever follows
  const int nkb = (kv_len + KVB - 1) / KVB;
  const long tail0 = (long)(nkb - 1) * KVB;  // first row of the last block
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.k + (long)kv_row0 * a.ks + h * D), (short)0, (int)(((long)kv_len - 1) * a.ks * 2 + 256), 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.v + (long)kv_row0 * a.vs + h * D), (short)0, (int)(((long)kv_len - 1) * a.vs * 2 + 256), 0x00020000);
  const __amdgpu_buffer_rsrc_t rkt = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.k + (kv_row0 + tail0) * a.ks + h * D), (short)0, (int)((kv_len - tail0 - 1) * a.ks * 2 + 256),
      0x00020000);
  const __amdgpu_buffer_rsrc_t rvt = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.v + (kv_row0 + tail0) * a.vs + h * D), (short)0, (int)((kv_len - tail0 - 1) * a.vs * 2 + 256),
      0x00020000);
  const bool ragged = kv_len % KVB != 0;
  int koff[PPW], voff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int srow = (wave * PPW + i) * 4 + (lane >> 4);
    koff[i] = srow * (int)a.ks * 2 + ((r16 ^ (srow & 15)) << 4);
    voff[i] = srow * (int)a.vs * 2 + ((r16 ^ ((srow & 7) << 1)) << 4);
  }
  const uint32_t lds_dma = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem) + wave * PPW * 1024);
  auto stage = [&](int kb, int buf) {
    const bool tail = ragged && kb == nkb - 1;  // wave-uniform
    const int ks_off = tail ? 0 : kb * KVB * (int)a.ks * 2, vs_off = tail ? 0 : kb * KVB * (int)a.vs * 2;
    const __amdgpu_buffer_rsrc_t bk = tail ? rkt : rk, bv = tail ? rvt : rv;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(bk, LDS_PTR((uintptr_t)(lds_dma + buf * STAGE_BYTES + i * 1024)), 16,
                                               koff[i], ks_off, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          bv, LDS_PTR((uintptr_t)(lds_dma + buf * STAGE_BYTES + TILE_BYTES + i * 1024)), 16, voff[i], vs_off, 0, 0);
    }
  };

  // per-lane LDS read bases (stage 0, key tile / chunk 0); the rest are +immediate
  const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(smem);
  uint32_t ka[4], va[8];
#pragma unroll
  for (int dc = 0; dc < 4; ++dc) ka[dc] = lds0 + r16 * 256 + (((dc * 4 + g) ^ r16) << 4);
  {
    const int q = r16 >> 2, p = r16 & 3;
    const int row = 4 * g + q;  // + 32 c (+16): same swizzle
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const int ch = 2 * dt + (p >> 1);
      va[dt] = lds0 + row * 256 + ((ch ^ ((row & 7) << 1)) << 4) + 8 * (p & 1);
    }
  }

  V6State st;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) st.O[dt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  st.L[0] = st.L[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  st.negm[0] = st.negm[1] = 0.f;
  st.negm4[0] = st.negm4[1] = (f32x4){0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  if (NW == 8 && __builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (1 < nkb) stage(1, 1);
  attn_v6_block<0, TILE_BYTES, true>(st, qf, ka, va, 0, kv_len, g);
  for (int kb = 1; kb < nkb; kb += 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kb + 1 < nkb) stage(kb + 1, 0);
    attn_v6_block<STAGE_BYTES, STAGE_BYTES + TILE_BYTES, false>(st, qf, ka, va, kb, kv_len, g);
    if (kb + 1 >= nkb) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kb + 2 < nkb) stage(kb + 2, 1);
    attn_v6_block<0, TILE_BYTES, false>(st, qf, ka, va, kb + 1, kv_len, g);
  }

  if (SPLIT && half >= 0) {  // partials: O^T[d][query] of this lane's d = 16 dt + 4 g + i, the query's max and sum
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int row = wave * 32 + qt * 16 + r16;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) *(f32x4*)(wblk + row * D + dt * 16 + 4 * g) = st.O[dt][qt];
      if (g == 0) {
        wblk[QBW * D + row] = -st.negm[qt];
        wblk[QBW * D + QBW + row] = st.L[qt][0];
      }
    }
    return;
  }
  // lane rows g and g^1 (lanes l, l^16) hold adjacent 4-column groups of one query row: one
  // permlane16 swap per dword pairs d tiles (dt, dt+1) so each lane stores 16 contiguous bytes (T21)
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const float inv = 1.0f / st.L[qt][0];
    const int qi = qb * QBW + wave * 32 + qt * 16 + r16;
    const int qrow = q_row0 + min(qi, q_len - 1);
    const int orow = a.orows ? a.orows[qrow] : qrow;
    bf16* op = a.o + (long)orow * a.os + h * D + 4 * (g & ~1) + 16 * (g & 1);
#pragma unroll
    for (int dt = 0; dt < 8; dt += 2) {
      const f32x4& A = st.O[dt][qt];
      const f32x4& B = st.O[dt + 1][qt];
      const bf16x4 pa = {f2bf(A[0] * inv), f2bf(A[1] * inv), f2bf(A[2] * inv), f2bf(A[3] * inv)};
      const bf16x4 pb = {f2bf(B[0] * inv), f2bf(B[1] * inv), f2bf(B[2] * inv), f2bf(B[3] * inv)};
      const u32x2 ga = __builtin_bit_cast(u32x2, pa), gb = __builtin_bit_cast(u32x2, pb);
      const auto rx = __builtin_amdgcn_permlane16_swap(ga[0], gb[0], false, false);
      const auto ry = __builtin_amdgcn_permlane16_swap(ga[1], gb[1], false, false);
      u32x4 out = {rx[0], ry[0], rx[1], ry[1]};
      bf16* p = op + dt * 16;
      if (a.accumulate) {  // bf16 + bf16 as the reference's sum of attention outputs (1B:602)
        const bf16x8 ov = *(const bf16x8*)p;
        bf16x8 nv = __builtin_bit_cast(bf16x8, out);
#pragma unroll
        for (int j = 0; j < 8; ++j) nv[j] = f2bf(bf2f(ov[j]) + bf2f(nv[j]));
        out = __builtin_bit_cast(u32x4, nv);
      }
      if (qi < q_len) *(u32x4*)p = out;
    }
  }
}

// self-attention reading V as V^T (attn_v6t_block above): 8 waves x 32 queries, the v6 ring and K staging.
// a.v = V^T [heads * 128][Rv] bf16 (row h*128 + d, keys permuted per 32 as P; a.vs = Rv >= the columns any
// segment's last 64-key block reaches, i.e. kv_row0 + ceil64(kv_len); segments start on 32-key boundaries; every
// element of a row readable and finite through that block: the partial last block reads the keys past kv_len,
// masked to P = 0).  2-stage K/V ring: block kb+1's DMA issued at block kb (one block of lead, vmcnt(0) +
// __syncthreads() per block).
__device__ __forceinline__ void attn_fwd_vt_body(const AttnArgs& a) {
  constexpr int NW = 8, QBW = NW * 32, PPW = 16 / NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nx = gridDim.x, ny = gridDim.y;
  const int flat = xcd_remap(blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z), nx * ny * gridDim.z);
  const int qb = flat % nx, h = (flat / nx) % ny, seg = flat / (nx * ny);
  const int* sg = a.segs + seg * 4;
  const int q_row0 = sg[0], q_len = sg[1], kv_row0 = sg[2], kv_len = sg[3];
  if (qb * QBW >= q_len) return;
  const int tid = threadIdx.x, lane = tid & 63;
  if (kv_len <= 0) {
    if (!a.accumulate)
      for (int i = tid; i < QBW * (D / 8); i += NW * 64) {
        const int qi = qb * QBW + i / (D / 8);
        if (qi < q_len) {
          const int orow = a.orows ? a.orows[q_row0 + qi] : q_row0 + qi;
          *(u32x4*)(a.o + (long)orow * a.os + h * D + (i % (D / 8)) * 8) = (u32x4){0u, 0u, 0u, 0u};
        }
      }
    return;
  }
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  bf16x8 qf[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qc = min(qb * QBW + wave * 32 + qt * 16 + r16, q_len - 1);
    const bf16* qp = a.q + (long)(q_row0 + qc) * a.qs + h * D + 8 * g;
#pragma unroll
    for (int dc = 0; dc < 4; ++dc) {
      qf[qt][dc] = *(const bf16x8*)(qp + 32 * dc);
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[qt][dc][j] = f2bf(bf2f(qf[qt][dc][j]) * a.c);
    }
  }
  const int nkb = (kv_len + KVB - 1) / KVB;
  const long tail0 = (long)(nkb - 1) * KVB;
  const bool ragged = kv_len % KVB != 0;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.k + (long)kv_row0 * a.ks + h * D), (short)0, (int)(((long)kv_len - 1) * a.ks * 2 + 256), 0x00020000);
  const __amdgpu_buffer_rsrc_t rkt = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.k + (kv_row0 + tail0) * a.ks + h * D), (short)0, (int)((kv_len - tail0 - 1) * a.ks * 2 + 256),
      0x00020000);
  // V^T: the head's 128 d-rows from key kv_row0, each through the segment's last block
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.v + (long)h * D * a.vs + kv_row0), (short)0, (int)(((long)(D - 1) * a.vs + (long)nkb * KVB) * 2),
      0x00020000);
  const int dw = wave;  // this wave's share of the K / V pieces
  int koff[PPW], voff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int srow = (dw * PPW + i) * 4 + (lane >> 4);
    koff[i] = srow * (int)a.ks * 2 + ((r16 ^ (srow & 15)) << 4);
    const int d = (dw * PPW + i) * 8 + (lane >> 3);  // a 1-KB piece = 8 d-rows x 128 B
    voff[i] = d * (int)a.vs * 2 + (((lane & 7) ^ (d & 7)) << 4);
  }
  const uint32_t lds_dma = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem) + dw * PPW * 1024);
  auto stage = [&](int kb, int buf) {  // LDS: 2 stages as K | V pairs
    const bool tail = ragged && kb == nkb - 1;
    const int ks_off = tail ? 0 : kb * KVB * (int)a.ks * 2, vs_off = kb * KVB * 2;
    const __amdgpu_buffer_rsrc_t bk = tail ? rkt : rk;
    const int kdst = buf * STAGE_BYTES, vdst = buf * STAGE_BYTES + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(bk, LDS_PTR((uintptr_t)(lds_dma + kdst + i * 1024)), 16, koff[i],
                                               ks_off, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, LDS_PTR((uintptr_t)(lds_dma + vdst + i * 1024)), 16, voff[i],
                                               vs_off, 0, 0);
    }
  };
  const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(smem);
  uint32_t ka[4], vb[2];
#pragma unroll
  for (int dc = 0; dc < 4; ++dc) ka[dc] = lds0 + r16 * 256 + (((dc * 4 + g) ^ r16) << 4);
#pragma unroll
  for (int c = 0; c < 2; ++c) vb[c] = lds0 + r16 * 128 + (((4 * c + g) ^ (r16 & 7)) << 4);

  V6State st;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) st.O[dt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  st.L[0] = st.L[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  st.negm[0] = st.negm[1] = 0.f;
  st.negm4[0] = st.negm4[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto sync = [] {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  stage(0, 0);
  if (__builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);
  sync();
  if (1 < nkb) stage(1, 1);
  attn_v6t_block<0, TILE_BYTES, true>(st, qf, ka, vb, 0, kv_len, g);
  for (int kb = 1; kb < nkb; kb += 2) {
    sync();
    if (kb + 1 < nkb) stage(kb + 1, 0);
    attn_v6t_block<STAGE_BYTES, STAGE_BYTES + TILE_BYTES, false>(st, qf, ka, vb, kb, kv_len, g);
    if (kb + 1 >= nkb) break;
    sync();
    if (kb + 2 < nkb) stage(kb + 2, 1);
    attn_v6t_block<0, TILE_BYTES, false>(st, qf, ka, vb, kb + 1, kv_len, g);
  }

#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const float inv = 1.0f / st.L[qt][0];
    const int qi = qb * QBW + wave * 32 + qt * 16 + r16;
    const int qrow = q_row0 + min(qi, q_len - 1);
    const int orow = a.orows ? a.orows[qrow] : qrow;
    bf16* op = a.o + (long)orow * a.os + h * D + 4 * (g & ~1) + 16 * (g & 1);
#pragma unroll
    for (int dt = 0; dt < 8; dt += 2) {
      const f32x4& A = st.O[dt][qt];
      const f32x4& B = st.O[dt + 1][qt];
      const bf16x4 pa = {f2bf(A[0] * inv), f2bf(A[1] * inv), f2bf(A[2] * inv), f2bf(A[3] * inv)};
      const bf16x4 pb = {f2bf(B[0] * inv), f2bf(B[1] * inv), f2bf(B[2] * inv), f2bf(B[3] * inv)};
      const u32x2 ga = __builtin_bit_cast(u32x2, pa), gb = __builtin_bit_cast(u32x2, pb);
      const auto rx = __builtin_amdgcn_permlane16_swap(ga[0], gb[0], false, false);
      const auto ry = __builtin_amdgcn_permlane16_swap(ga[1], gb[1], false, false);
      u32x4 out = {rx[0], ry[0], rx[1], ry[1]};
      bf16* p = op + dt * 16;
      if (a.accumulate) {
        const bf16x8 ov = *(const bf16x8*)p;
        bf16x8 nv = __builtin_bit_cast(bf16x8, out);
#pragma unroll
        for (int j = 0; j < 8; ++j) nv[j] = f2bf(bf2f(ov[j]) + bf2f(nv[j]));
        out = __builtin_bit_cast(u32x4, nv);
      }
      if (qi < q_len) *(u32x4*)p = out;
    }
  }
}

// the fused cross-attention on the self-attention block body: 8 waves x 32 queries of one query block,
// the text, image and per-frame vocal K/V streams one after the other through 3-stage K / V regions (each
// block's DMA two blocks ahead), a separate online softmax per source (its first block sets the max), the
// three bf16 outputs summed as the reference does
// NW waves x 32 queries per workgroup, NST-stage K / V ring (block j's DMA NST - 1 blocks ahead)
template <int NW, int NST>
__device__ __forceinline__ void attn_cross3_body(const Cross3Args& a) {
  constexpr int QBW = NW * 32, PPW = 16 / NW;  // queries per workgroup, K (and V) 1-KB pieces per wave per block
  constexpr int VBASE = NST * TILE_BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nx = gridDim.x, ny = gridDim.y;
  const int flat = xcd_remap(blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z), nx * ny * gridDim.z);
  const int qb = flat % nx, h = (flat / nx) % ny, b = flat / (nx * ny);
  if (qb * QBW >= a.q_len) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int q_row0 = b * a.q_len;
  const int frame = (a.tok_offset + qb * QBW) / a.tpf;

  // Q as the B operand (query tile qt, d chunk dc), prescaled by c; rows clamped to the segment
  bf16x8 qf[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qc = min(qb * QBW + wave * 32 + qt * 16 + r16, a.q_len - 1);
    const bf16* qp = a.q + (long)(q_row0 + qc) * a.qs + h * D + 8 * g;
#pragma unroll
    for (int dc = 0; dc < 4; ++dc) {
      qf[qt][dc] = *(const bf16x8*)(qp + 32 * dc);
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[qt][dc][j] = f2bf(bf2f(qf[qt][dc][j]) * a.c);
    }
  }

  // block stream: text blocks, image blocks, vocal block(s); LDS images as the self-attention kernel's
  // (K rows chunk ^ (row & 15), V rows chunk ^ 2 (row & 7)); each wave moves 2 x 1-KB pieces of K and V
  const int nT = (a.t_len + KVB - 1) / KVB, nI = (a.i_len + KVB - 1) / KVB, nV = (a.nper + KVB - 1) / KVB;
  const int ntot = nT + nI + nV;
  // staging by buffer descriptors rebased per block (SALU: base = the block's first row of this batch row's
  // source, range = its rows up to the source's last), so rows past the source read as zeros and are masked;
  // per-lane 32-bit offsets -- no 64-bit address VALU per block (the round-3 kernel formed clamped 64-bit row
  // addresses for every piece of every block).  The rows past a source's last key (the image stream's last block:
  // 257 = 4 x 64 + 1 keys) read as zeros through the records bound (the range check counts soffset too, round 6)
  int srow[PPW], kch[PPW], vch[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    srow[i] = (wave * PPW + i) * 4 + (lane >> 4);
    kch[i] = r16 ^ (srow[i] & 15);
    vch[i] = r16 ^ ((srow[i] & 7) << 1);
  }
  const long vrow0 = (long)(b * a.n_frames + frame) * a.nper;
  const bf16* const kt0 = a.kt + (long)b * a.t_len * a.ts + h * D;
  const bf16* const vt0 = a.vt + (long)b * a.t_len * a.ts + h * D;
  const bf16* const ki0 = a.ki + (long)b * a.i_len * a.is + h * D;
  const bf16* const vi0 = a.vi + (long)b * a.i_len * a.is + h * D;
  const bf16* const kv0 = a.kv + vrow0 * a.vs + h * D;
  const bf16* const vv0 = a.vv + vrow0 * a.vs + h * D;
  const uint32_t lds_k = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem) + wave * PPW * 1024);
  auto stage = [&](int j, int buf) {
    const bf16 *kb0 = kt0, *vb0 = vt0;
    int st = (int)a.ts, blk = j, len = a.t_len;
    if (j >= nT + nI) {
      kb0 = kv0; vb0 = vv0; st = (int)a.vs; blk = j - nT - nI; len = a.nper;
    } else if (j >= nT) {
      kb0 = ki0; vb0 = vi0; st = (int)a.is; blk = j - nT; len = a.i_len;
    }
    const long r0 = (long)blk * KVB;
    const int nrec = (int)((min((long)len - r0, (long)KVB) - 1) * st * 2 + 256);
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void*)(kb0 + r0 * st), (short)0, nrec, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)(vb0 + r0 * st), (short)0, nrec, 0x00020000);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int rowoff = srow[i] * st * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, LDS_PTR((uintptr_t)(lds_k + buf * TILE_BYTES + i * 1024)), 16,
                                               rowoff + kch[i] * 16, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rv, LDS_PTR((uintptr_t)(lds_k + VBASE + buf * TILE_BYTES + i * 1024)), 16, rowoff + vch[i] * 16, 0, 0, 0);
    }
  };

  const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(smem);
  uint32_t ka[4], va[8];
#pragma unroll
  for (int dc = 0; dc < 4; ++dc) ka[dc] = lds0 + r16 * 256 + (((dc * 4 + g) ^ r16) << 4);
  {
    const int q4 = r16 >> 2, p4 = r16 & 3;
    const int row = 4 * g + q4;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const int ch = 2 * dt + (p4 >> 1);
      va[dt] = lds0 + VBASE + row * 256 + ((ch ^ ((row & 7) << 1)) << 4) + 8 * (p4 & 1);
    }
  }

  V6State st;
  auto reset = [&]() {
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) st.O[dt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    st.L[0] = st.L[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
    st.negm[0] = st.negm[1] = 0.f;
    st.negm4[0] = st.negm4[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  };
  reset();
  bf16x4 acc[8][2];  // running (text + img) + vocal, bf16 as in the reference
  // finish source `src` (0 text, 1 image, 2 vocal): bf16(O / l) folded into acc
  auto finish = [&](int src) {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float inv = 1.0f / st.L[qt][0];
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        bf16x4 x;
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = f2bf(st.O[dt][qt][i] * inv);
        if (src == 0) {
          acc[dt][qt] = x;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[dt][qt][i] = f2bf(bf2f(acc[dt][qt][i]) + bf2f(x[i]));
        }
      }
    }
    reset();
  };

  // Block j sits in ring slot j % NST, chosen at run time through the LDS read bases (kas / vas): one copy of the
  // block body.  With a copy per slot (the slot as the ds_read immediate offset, round 4) hipcc spilled 118 (8 waves)
  // / 152 (4 waves) VGPRs to scratch: every copy's temporaries live across the unrolled loop.
  uint32_t kas[4], vas[8];
  auto at_slot = [&](int slot) {
    const uint32_t so = (uint32_t)slot * TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) kas[i] = ka[i] + so;
#pragma unroll
    for (int i = 0; i < 8; ++i) vas[i] = va[i] + so;
  };
  // block j's DMA issued NST - 1 blocks ahead (with one block of lead the L2 latency of the next block was exposed
  // at the barriers of these short streams)
  auto step = [&](int jj) {
    if (NST > 2 && jj + 1 < ntot)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PPW) : "memory");  // block jj landed; jj+1 may still fly
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (jj + NST - 1 < ntot) stage(jj + NST - 1, (jj + NST - 1) % NST);
    const int src = jj < nT ? 0 : (jj < nT + nI ? 1 : 2);
    const int kb = src == 0 ? jj : (src == 1 ? jj - nT : jj - nT - nI);
    const int len = src == 0 ? a.t_len : (src == 1 ? a.i_len : a.nper);
    at_slot(jj % NST);
    attn_v6_block<0, 0, false, false>(st, qf, kas, vas, kb, len, g, kb == 0);
    if (jj == nT - 1 || jj == nT + nI - 1 || jj == ntot - 1) finish(src);
  };
  // the vocal stream's single block when a frame has at most 32 audio tokens (StableAvatar: 32), and the image
  // stream's last block when it holds at most 32 keys (CLIP: 257 = 4 x 64 + 1) while the vocal block is peeled too:
  // peeled out of the loop as half blocks (key tiles 0-1: half the MFMAs and exponentials of a 64-key block)
  const bool vhalf = nV == 1 && a.nper <= KVB / 2;
  const bool ihalf = vhalf && a.i_len % KVB != 0 && a.i_len % KVB <= KVB / 2;
  auto half = [&](bool voc) {
    const int jj = voc ? ntot - 1 : ntot - 2;
    if (!voc && NST > 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PPW) : "memory");  // this block landed; the vocal block may fly
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (!voc && NST == 2) stage(jj + 1, (jj + 1) % NST);  // the vocal block, one ahead
    at_slot(jj % NST);
    attn_half_block<0, 0>(st, qf, kas, vas, voc ? 0 : nI - 1, voc ? a.nper : a.i_len, g, voc || nI == 1);
    finish(voc ? 2 : 1);
  };
  const int nloop = vhalf ? (ihalf ? ntot - 2 : ntot - 1) : ntot;
  if (NW == 8 && __builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);
  stage(0, 0);
  if (NST > 2 && 1 < ntot) stage(1, 1);
  for (int j = 0; j < nloop; ++j) step(j);
  for (int hb = ihalf ? 0 : 1; hb < (vhalf ? 2 : 0); ++hb) half(hb == 1);

  // 16-byte stores from permlane16-swapped column-group pairs, as the self-attention epilogue (T21)
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = qb * QBW + wave * 32 + qt * 16 + r16;
    bf16* op = a.o + (long)(q_row0 + min(qi, a.q_len - 1)) * a.os + h * D + 4 * (g & ~1) + 16 * (g & 1);
#pragma unroll
    for (int dt = 0; dt < 8; dt += 2) {
      const u32x2 ga = __builtin_bit_cast(u32x2, acc[dt][qt]), gb = __builtin_bit_cast(u32x2, acc[dt + 1][qt]);
      const auto rx = __builtin_amdgcn_permlane16_swap(ga[0], gb[0], false, false);
      const auto ry = __builtin_amdgcn_permlane16_swap(ga[1], gb[1], false, false);
      if (qi < a.q_len) *(u32x4*)(op + dt * 16) = (u32x4){rx[0], ry[0], rx[1], ry[1]};
    }
  }
}

__global__ __launch_bounds__(512) void attn_cross3_kernel(Cross3Args a) { attn_cross3_body<8, 3>(a); }
// 4 waves x 32 queries, 2-stage ring (64 KB): two workgroups per CU, so one's prologue (Q from HBM) and epilogue
// stores run beside the other's blocks
__global__ __launch_bounds__(256, 2) void attn_cross3_w4_kernel(Cross3Args a) { attn_cross3_body<4, 2>(a); }

__global__ __launch_bounds__(512) void attn_fwd_v6_kernel(AttnArgs a) { attn_fwd_v6_body<8>(a); }
__global__ __launch_bounds__(512) void attn_fwd_v6_split_kernel(AttnArgs a) { attn_fwd_v6_body<8, true>(a); }

// the two key halves of each split tile -> the output: O = (w0 O0 + w1 O1) / (w0 l0 + w1 l1), w = 2^(m - max(m0, m1))
__global__ __launch_bounds__(256) void attn_split_merge_kernel(AttnArgs a) {
  const int stile = blockIdx.x, tile = a.split_full + stile;
  const int qb = tile % a.nqb, h = (tile / a.nqb) % a.nheads, seg = tile / (a.nqb * a.nheads);
  const int* sg = a.segs + seg * 4;
  const int q_row0 = sg[0], q_len = sg[1];
  if (qb * QB >= q_len) return;
  const float* w0 = a.work + (long)stile * 2 * QB * (D + 2);
  const float* w1 = w0 + QB * (D + 2);
  for (int i = threadIdx.x; i < QB * (D / 4); i += 256) {
    const int row = i / (D / 4), d = (i % (D / 4)) * 4, qi = qb * QB + row;
    if (qi >= q_len) continue;
    const float m0 = w0[QB * D + row], m1 = w1[QB * D + row];
    const float M = fmaxf(m0, m1);
    const float a0 = m0 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m0 - M);
    const float a1 = m1 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m1 - M);
    const float inv = 1.0f / (a0 * w0[QB * D + QB + row] + a1 * w1[QB * D + QB + row]);
    const f32x4 x0 = *(const f32x4*)(w0 + row * D + d), x1 = *(const f32x4*)(w1 + row * D + d);
    const int orow = a.orows ? a.orows[q_row0 + qi] : q_row0 + qi;
    bf16* p = a.o + (long)orow * a.os + h * D + d;
    bf16x4 o4;
#pragma unroll
    for (int j = 0; j < 4; ++j) o4[j] = f2bf((a0 * x0[j] + a1 * x1[j]) * inv);
    if (a.accumulate) {
      const bf16x4 ov = *(const bf16x4*)p;
#pragma unroll
      for (int j = 0; j < 4; ++j) o4[j] = f2bf(bf2f(ov[j]) + bf2f(o4[j]));
    }
    *(bf16x4*)p = o4;
  }
}
__global__ __launch_bounds__(256, 2) void attn_fwd_v6_w4_kernel(AttnArgs a) { attn_fwd_v6_body<4>(a); }
__global__ __launch_bounds__(512) void attn_fwd_v6t_kernel(AttnArgs a) { attn_fwd_vt_body(a); }

}  // namespace

// kernel: 0 = auto, 1 = attn_fwd_v6_kernel (8 waves x 32 queries, mfma_f32_16x16x32_bf16), 2 = the 4-wave
// attn_fwd_v6_w4_kernel (two workgroups per CU).  Auto estimates both launches in rounds of one 8-wave
// workgroup per CU: a 4-wave round holds two workgroups per CU and runs 3 % slower per FLOP; a last 4-wave
// round of at most one workgroup per CU (one wave per SIMD) takes 0.75 of a round (measured,
// profiles/r02/attn_sp_shapes.json: the Ulysses N = 8 shape, 378 / 756 workgroups, 1.036 vs 0.927 ms).
// o_rows (optional, device int32 indexed by query row): query row r's output goes to row o_rows[r] of o --
// the sequence-parallel path writes this rank's own token chunk straight into the O-projection's input
// panels and the other chunks into their send slabs (stableavatar_amd/sp.py)
extern "C" int sa_attn_fwd_map(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg,
                               int max_q_len, int heads, int head_dim, int64_t q_stride, int64_t k_stride,
                               int64_t v_stride, int64_t o_stride, float scale, int accumulate, int kernel,
                               const int32_t* o_rows, void* stream) {
  if (!q || !k || !v || !o || !segs || nseg <= 0 || max_q_len <= 0 || heads <= 0) return SA_ERR_ARG;
  if (head_dim != D) return SA_ERR_ARG;
  if ((q_stride | k_stride | v_stride | o_stride) % 8) return SA_ERR_ARG;
  if ((((uintptr_t)q) | ((uintptr_t)k) | ((uintptr_t)v) | ((uintptr_t)o)) & 15) return SA_ERR_ARG;
  if (kernel < 0 || kernel > 3) return SA_ERR_ARG;
  if (kernel == 3 && (v_stride % 64 || (((uintptr_t)v) & 127))) return SA_ERR_ARG;  // V^T rows: whole 64-key blocks
  static const bool attr = [] {  // one-time, thread-safe
    (void)hipFuncSetAttribute((const void*)attn_fwd_v6_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)attn_fwd_v6_w4_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)attn_fwd_v6t_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    return true;
  }();
  (void)attr;
  AttnArgs a{(const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, segs,
             q_stride, k_stride, v_stride, o_stride, scale * 1.4426950408889634f, accumulate, o_rows};
  if (kernel == 0) {
    static int cus[64] = {0};  // per device, queried once
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
      if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus[dev] = 256;
      ncu = cus[dev] > 0 ? cus[dev] : 256;
    }
    const long n8 = (long)nseg * heads * ((max_q_len + 255) / 256), n4 = (long)nseg * heads * ((max_q_len + 127) / 128);
    const long t8 = (n8 + ncu - 1) / ncu, full = n4 / (2 * ncu), rem = n4 % (2 * ncu);
    const double t4 = 1.03 * (full + (rem == 0 ? 0.0 : (rem <= ncu ? 0.75 : 1.0)));
    kernel = t4 < (double)t8 ? 2 : 1;
  }
  if (kernel == 2) {
    dim3 grid((max_q_len + 127) / 128, heads, nseg);
    hipLaunchKernelGGL(attn_fwd_v6_w4_kernel, grid, dim3(256), LDS_BYTES, (hipStream_t)stream, a);
  } else if (kernel == 3) {  // v = V^T [heads * 128][v_stride] (attn_fwd_vt_body)
    dim3 grid((max_q_len + QB - 1) / QB, heads, nseg);
    hipLaunchKernelGGL(attn_fwd_v6t_kernel, grid, dim3(512), LDS_BYTES, (hipStream_t)stream, a);
  } else {
    dim3 grid((max_q_len + QB - 1) / QB, heads, nseg);
    hipLaunchKernelGGL(attn_fwd_v6_kernel, grid, dim3(512), LDS_BYTES, (hipStream_t)stream, a);
  }
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_attn_fwd_split(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg,
                                 int max_q_len, int heads, int head_dim, int64_t q_stride, int64_t k_stride,
                                 int64_t v_stride, int64_t o_stride, float scale, int accumulate, const int32_t* o_rows,
                                 int split_tiles, void* work, int64_t work_bytes, void* stream) {
  if (!q || !k || !v || !o || !segs || nseg <= 0 || max_q_len <= 0 || heads <= 0 || head_dim != D) return SA_ERR_ARG;
  if ((q_stride | k_stride | v_stride | o_stride) % 8) return SA_ERR_ARG;
  if ((((uintptr_t)q) | ((uintptr_t)k) | ((uintptr_t)v) | ((uintptr_t)o)) & 15) return SA_ERR_ARG;
  const int nqb = (max_q_len + QB - 1) / QB;
  const long ntiles = (long)nseg * heads * nqb;
  if (split_tiles <= 0 || split_tiles > ntiles) return SA_ERR_ARG;
  if (!work || (((uintptr_t)work) & 15) || work_bytes < (int64_t)split_tiles * 2 * QB * (D + 2) * 4) return SA_ERR_ARG;
  static const bool attr = [] {
    (void)hipFuncSetAttribute((const void*)attn_fwd_v6_split_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES);
    return true;
  }();
  (void)attr;
  AttnArgs a{(const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, segs,
             q_stride, k_stride, v_stride, o_stride, scale * 1.4426950408889634f, accumulate, o_rows,
             nqb, heads, (int)(ntiles - split_tiles), split_tiles, (float*)work};
  hipLaunchKernelGGL(attn_fwd_v6_split_kernel, dim3((unsigned)(ntiles + split_tiles)), dim3(512), LDS_BYTES,
                     (hipStream_t)stream, a);
  SA_LAUNCH_CHECK();
  hipLaunchKernelGGL(attn_split_merge_kernel, dim3(split_tiles), dim3(256), 0, (hipStream_t)stream, a);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_attn_fwd_ex(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg,
                              int max_q_len, int heads, int head_dim, int64_t q_stride, int64_t k_stride,
                              int64_t v_stride, int64_t o_stride, float scale, int accumulate, int kernel,
                              void* stream) {
  return sa_attn_fwd_map(q, k, v, o, segs, nseg, max_q_len, heads, head_dim, q_stride, k_stride, v_stride, o_stride,
                         scale, accumulate, kernel, nullptr, stream);
}

extern "C" int sa_attn_fwd(const void* q, const void* k, const void* v, void* o, const int32_t* segs, int nseg,
                           int max_q_len, int heads, int head_dim, int64_t q_stride, int64_t k_stride,
                           int64_t v_stride, int64_t o_stride, float scale, int accumulate, void* stream) {
  return sa_attn_fwd_ex(q, k, v, o, segs, nseg, max_q_len, heads, head_dim, q_stride, k_stride, v_stride, o_stride,
                        scale, accumulate, 0, stream);
}

extern "C" int sa_attn_cross3(const void* q, int64_t q_stride, const void* kt, const void* vt, int64_t t_stride,
                              int t_len, const void* ki, const void* vi, int64_t i_stride, int i_len, const void* kv,
                              const void* vv, int64_t v_stride, int nper, int tokens_per_frame, int n_frames,
                              int tok_offset, void* o, int64_t o_stride, int batch, int q_len, int heads,
                              float scale, void* stream) {
  if (!q || !kt || !vt || !ki || !vi || !kv || !vv || !o) return SA_ERR_ARG;
  if (batch <= 0 || q_len <= 0 || heads <= 0 || t_len <= 0 || i_len <= 0 || nper <= 0 || n_frames <= 0)
    return SA_ERR_ARG;
  if (tokens_per_frame <= 0 || tokens_per_frame % QB != 0 || tok_offset < 0 || tok_offset % QB != 0 ||
      (long)n_frames * tokens_per_frame < (long)tok_offset + q_len)
    return SA_ERR_ARG;
  if ((q_stride | t_stride | i_stride | v_stride | o_stride) % 8) return SA_ERR_ARG;
  if ((((uintptr_t)q) | ((uintptr_t)kt) | ((uintptr_t)vt) | ((uintptr_t)ki) | ((uintptr_t)vi) | ((uintptr_t)kv) |
       ((uintptr_t)vv) | ((uintptr_t)o)) & 15)
    return SA_ERR_ARG;
  static const bool attr = [] {
    (void)hipFuncSetAttribute((const void*)attn_cross3_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, X3_LDS);
    (void)hipFuncSetAttribute((const void*)attn_cross3_w4_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              4 * TILE_BYTES);
    return true;
  }();
  (void)attr;
  Cross3Args a{(const bf16*)q, q_stride, (const bf16*)kt, (const bf16*)vt, t_stride, t_len, (const bf16*)ki,
               (const bf16*)vi, i_stride, i_len, (const bf16*)kv, (const bf16*)vv, v_stride, nper,
               tokens_per_frame, n_frames, tok_offset, (bf16*)o, o_stride, q_len, scale * 1.4426950408889634f};
  // 4-wave workgroups, two per CU (0.369-0.377 vs 0.390 ms per config-2 launch, same output; SA_X3_W4=0: 8 waves)
  const char* w4 = getenv("SA_X3_W4");
  if (!w4 || atoi(w4)) {
    dim3 grid((q_len + 127) / 128, heads, batch);
    hipLaunchKernelGGL(attn_cross3_w4_kernel, grid, dim3(256), 4 * TILE_BYTES, (hipStream_t)stream, a);
  } else {
    dim3 grid((q_len + QB - 1) / QB, heads, batch);
    hipLaunchKernelGGL(attn_cross3_kernel, grid, dim3(512), X3_LDS, (hipStream_t)stream, a);
  }
  SA_LAUNCH_CHECK();
  return SA_OK;
}
