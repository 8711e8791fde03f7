// Row normalisations of the DiT / vocal projector, one wave per row, fp32 math:
//  * sa_layernorm_mod: LayerNorm (biased var, eps) -> optional affine -> optional AdaLN
//    modulate  y*(1+scale[b]) + shift[b]                      (1B:345-355,675,684,687,721-722;
//    vocal_projector_fantasy_1B.py:345,352,354,386,398; MLPProj 1B:731-734)
//    and an optional gated residual  out = x + y*gate[b]       (vocal_projector_fantasy_1B.py:345-347)
//  * sa_qk_rmsnorm_rope: WanRMSNorm over the FULL model dim on q and k (1B:326-342,395-396),
//    then the 3-D complex RoPE (1B:295-323) with fp64-derived fp32 (cos,sin) tables; tokens past
//    f*h*w (padding) are left unrotated (1B:319).  In place on the fused QKV GEMM output.
#include "common.h"
#include <cstdlib>

#ifndef SA_LN_SHARED_DEFAULT
#define SA_LN_SHARED_DEFAULT 8
#endif

namespace {

template <typename TI>
__device__ __forceinline__ void load8(const TI* p, float* v);
template <>
__device__ __forceinline__ void load8<float>(const float* p, float* v) {
  f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
template <>
__device__ __forceinline__ void load8<bf16>(const bf16* p, float* v) {
  bf16x8 a = *(const bf16x8*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f(a[j]);
}
template <typename TO>
__device__ __forceinline__ void store8(TO* p, const float* v);
template <>
__device__ __forceinline__ void store8<float>(float* p, const float* v) {
  *(f32x4*)p = (f32x4){v[0], v[1], v[2], v[3]};
  *(f32x4*)(p + 4) = (f32x4){v[4], v[5], v[6], v[7]};
}
template <>
__device__ __forceinline__ void store8<bf16>(bf16* p, const float* v) {
  bf16x8 a;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = f2bf(v[j]);
  *(bf16x8*)p = a;
}

struct LnArgs {
  const void* x; long ldx;
  void* out; long ldo;
  const float* w; const float* b;         // affine (optional)
  const float* shift; const float* scale; long mod_bstride;  // AdaLN (optional)
  const float* gate;                       // gated residual (optional, f32 out only)
  int rows_per_batch;
  int M, C;
  float eps;
};

constexpr int MAXV = 10;  // up to 10 chunks of 8 per lane -> C <= 5120 (the 14B DiT width)

// FIXED > 0: C == FIXED * 512 known at compile time (the DiT's C = 1536), so every chunk's loads are
// unconditional and issue together; FIXED == 0: any C % 8 == 0 up to 5120.
template <typename TI, typename TO, int FIXED = 0>
__global__ __launch_bounds__(256) void layernorm_mod_kernel(LnArgs a) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.M) return;
  const TI* x = (const TI*)a.x + (long)row * a.ldx;
  const int nch = FIXED ? FIXED : (a.C + 511) / 512;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (i < nch && (FIXED || i * 512 + lane * 8 < a.C)) {
      load8<TI>(x + i * 512 + lane * 8, v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  const float mean = wave_sum(s) / a.C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (i < nch && (FIXED || i * 512 + lane * 8 < a.C)) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; q = __builtin_fmaf(d, d, q); }
    }
  const float rstd = rsqrtf(wave_sum(q) / a.C + a.eps);
  const long bo = (long)(row / a.rows_per_batch) * a.mod_bstride;
  TO* out = (TO*)a.out + (long)row * a.ldo;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (i < nch && (FIXED || i * 512 + lane * 8 < a.C)) {
      const int c0 = i * 512 + lane * 8;
      float y[8], w8[8], b8[8], sc8[8], sh8[8], g8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = (v[i][j] - mean) * rstd;
      if (a.w) {
        load8<float>(a.w + c0, w8);
        if (a.b) load8<float>(a.b + c0, b8);
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = __builtin_fmaf(y[j], w8[j], a.b ? b8[j] : 0.f);
      }
      if (a.scale) {
        load8<float>(a.scale + bo + c0, sc8);
        load8<float>(a.shift + bo + c0, sh8);
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = __builtin_fmaf(y[j], 1.f + sc8[j], sh8[j]);
      }
      if (a.gate) {
        load8<float>(a.gate + bo + c0, g8);
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = __builtin_fmaf(y[j], g8[j], v[i][j]);
      }
      store8<TO>(out + c0, y);
    }
}

struct QkArgs {
  bf16* x; long ldx;
  int q_col, k_col;  // column offsets of q and k inside a row (k_col < 0: q only)
  const float* wq; const float* wk;
  int M, C, head_dim;
  float eps;
  const float* rope;  // [1024][head_dim/2][2] (cos, sin) or null
  int rows_per_batch, tok_offset, F, H, W;  // token t = tok_offset + row % rows_per_batch
  int nf, nh;         // pairs assigned to frame / height axes (rest: width)
};

// in-place store of one normalised 8-column chunk (c0 = column inside q or k)
struct StoreInPlace {
  bf16* p;
  __device__ __forceinline__ void operator()(int c0, const float* y) const { store8<bf16>(p + c0, y); }
};

template <int FIXED, class Store>
__device__ __forceinline__ void rms_rope_one(const bf16* p, const float* w, const QkArgs& a, int lane, int fi, int hi_,
                                             int wi, bool rot, const Store& store) {
  // explicit FMAs, no compiler contraction: the in-place and the SP pack instantiations round identically
#pragma clang fp contract(off)
  const int nch = FIXED ? FIXED : (a.C + 511) / 512;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (i < nch && (FIXED || i * 512 + lane * 8 < a.C)) {
      load8<bf16>(p + i * 512 + lane * 8, v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s = fmaf(v[i][j], v[i][j], s);
    }
  const float r = rsqrtf(wave_sum(s) / a.C + a.eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (i < nch && (FIXED || i * 512 + lane * 8 < a.C)) {
      const int c0 = i * 512 + lane * 8;
      float y[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = v[i][j] * r;
      {
        float w8[8];
        load8<float>(w + c0, w8);
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] *= w8[j];
      }
      if (rot) {
        const int d0 = c0 % a.head_dim;
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const int pi = (d0 + j) >> 1;
          const int pos = pi < a.nf ? fi : (pi < a.nf + a.nh ? hi_ : wi);
          const float2 csn = *(const float2*)(a.rope + (pos * (a.head_dim / 2) + pi) * 2);
          const float cs = csn.x, sn = csn.y;
          const float re = y[j], im = y[j + 1];
          y[j] = fmaf(re, cs, -(im * sn));
          y[j + 1] = fmaf(re, sn, im * cs);
        }
      }
      store(c0, y);
    }
}

template <int FIXED = 0>
__global__ __launch_bounds__(256) void qk_rmsnorm_rope_kernel(QkArgs a) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.M) return;
  bool rot = false;
  int fi = 0, hi_ = 0, wi = 0;
  if (a.rope) {
    const int t = a.tok_offset + row % a.rows_per_batch;
    if (t < a.F * a.H * a.W) {
      rot = true;
      fi = t / (a.H * a.W);
      hi_ = (t / a.W) % a.H;
      wi = t % a.W;
    }
  }
  bf16* base = a.x + (long)row * a.ldx;
  rms_rope_one<FIXED>(base + a.q_col, a.wq, a, lane, fi, hi_, wi, rot, StoreInPlace{base + a.q_col});
  if (a.k_col >= 0) rms_rope_one<FIXED>(base + a.k_col, a.wk, a, lane, fi, hi_, wi, rot, StoreInPlace{base + a.k_col});
}

// Self-attention case (C = 1536 = 3 x 512, head_dim 128, q and k, 3-D RoPE): one wave per token row
// loads q and k together (six 16-byte loads in flight), reduces both sums of squares in one
// butterfly, and applies RoPE with this lane's 4 (cos, sin) pairs, which are the same for every
// head chunk of the row ((i*512 + lane*8) % 128 does not depend on i) and for q and k.
__device__ __forceinline__ float2 wave_sum2(float2 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v.x += __shfl_xor(v.x, o, 64);
    v.y += __shfl_xor(v.y, o, 64);
  }
  return v;
}

// store(i, yq, yk): chunk i (columns i*512 + lane*8 .. +7) of the normalised, rotated q and k
template <class Store>
__device__ __forceinline__ void qk_pair_row(const QkArgs& a, int row, int lane, const Store& store) {
#pragma clang fp contract(off)  // explicit FMAs only (as rms_rope_one)
  constexpr int NCH = 3, HD = 128;
  const bf16* qp = a.x + (long)row * a.ldx + a.q_col + lane * 8;
  const bf16* kp = a.x + (long)row * a.ldx + a.k_col + lane * 8;
  float q[NCH][8], k[NCH][8];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    load8<bf16>(qp + i * 512, q[i]);
    load8<bf16>(kp + i * 512, k[i]);
  }
  float cs[4], sn[4];
  const int t = a.tok_offset + row % a.rows_per_batch;
  const bool rot = t < a.F * a.H * a.W;
  {
    const int fi = t / (a.H * a.W), hi_ = (t / a.W) % a.H, wi = t % a.W;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pi = ((lane * 8) % HD) / 2 + j;
      const int pos = pi < a.nf ? fi : (pi < a.nf + a.nh ? hi_ : wi);
      const float2 c = rot ? *(const float2*)(a.rope + (pos * (HD / 2) + pi) * 2) : make_float2(1.f, 0.f);
      cs[j] = c.x;
      sn[j] = c.y;
    }
  }
  float2 ss = make_float2(0.f, 0.f);
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ss.x = fmaf(q[i][j], q[i][j], ss.x);
      ss.y = fmaf(k[i][j], k[i][j], ss.y);
    }
  ss = wave_sum2(ss);
  const float rq = rsqrtf(ss.x / (NCH * 512) + a.eps), rk = rsqrtf(ss.y / (NCH * 512) + a.eps);
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c0 = i * 512 + lane * 8;
    float wq[8], wk[8], yq[8], yk[8];
    load8<float>(a.wq + c0, wq);
    load8<float>(a.wk + c0, wk);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      yq[j] = q[i][j] * rq * wq[j];
      yk[j] = k[i][j] * rk * wk[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float qr = yq[2 * j], qi = yq[2 * j + 1], kr = yk[2 * j], ki = yk[2 * j + 1];
      yq[2 * j] = fmaf(qr, cs[j], -(qi * sn[j]));
      yq[2 * j + 1] = fmaf(qr, sn[j], qi * cs[j]);
      yk[2 * j] = fmaf(kr, cs[j], -(ki * sn[j]));
      yk[2 * j + 1] = fmaf(kr, sn[j], ki * cs[j]);
    }
    store(i, yq, yk);
  }
}

__global__ __launch_bounds__(256) void qk_rmsnorm_rope_pair_kernel(QkArgs a) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.M) return;
  bf16* qp = a.x + (long)row * a.ldx + a.q_col + lane * 8;
  bf16* kp = a.x + (long)row * a.ldx + a.k_col + lane * 8;
  qk_pair_row(a, row, lane, [&](int i, const float* yq, const float* yk) {
    store8<bf16>(qp + i * 512, yq);
    store8<bf16>(kp + i * 512, yk);
  });
}

// ---- the Ulysses send-slab pack (replaces the torch.cat packing around
// wan/dist/wan_xfuser.py:72-115): the same per-row q/k RMSNorm + RoPE as above on the fused QKV GEMM
// output of this rank's token chunk, written -- with v -- straight into per-destination slabs instead of
// back in place.  Head group g (columns g*C/G .. of q, k and v) of token t in CFG row b goes to
//   q:    destination my_part*G + g (the rank that runs attention for this chunk's query part), and
//   k, v: destinations r*G + g for every query part r (each of them attends over all keys),
// entry d of the device table {q_ptr, q_ld, q_bstride, kv_ptr, kv_ld, kv_bstride} (elements; q_ptr 0 =
// no query slab for d): q row at q_ptr + b*q_bstride + t*q_ld, k at kv_ptr + b*kv_bstride + t*kv_ld, v at
// k + C/G.  The entry of this rank itself points into its own attention inputs, the others into the send
// buffers of the point-to-point exchange, so the pack is the only copy of Q/K/V on the way.
struct PackArgs {
  QkArgs qk;             // x = the [M, 3C] QKV rows (q at column 0, k at C, v at 2C)
  const long* table;     // [G*R][6]
  int G, R, my_part;
  int b_offset;          // CFG row of launch row 0 is b_offset + row / rows_per_batch
};

struct PackStore {
  const long* table;
  int G, R, my_part, hgd;
  long b, t;
  const bf16* vrow;  // this row's v
  template <bool Q>
  __device__ __forceinline__ void put(int c0, const float* y) const {
    const int g = c0 / hgd, w = c0 - g * hgd;
    if (Q) {
      const long* e = table + (long)(my_part * G + g) * 6;
      store8<bf16>((bf16*)e[0] + b * e[2] + t * e[1] + w, y);
    } else {
      // k | v once, into this query part's entry of head group g: the exchange sends that slab to the group's rank
      // of every query part (the K/V of a group is the same for all of them)
      const u32x4 vv = *(const u32x4*)(vrow + c0);
      const long* e = table + (long)(my_part * G + g) * 6;
      bf16* kd = (bf16*)e[3] + b * e[5] + t * e[4] + w;
      store8<bf16>(kd, y);
      *(u32x4*)(kd + hgd) = vv;
    }
  }
};

template <bool Q>
struct PackOne {
  const PackStore* ps;
  __device__ __forceinline__ void operator()(int c0, const float* y) const { ps->put<Q>(c0, y); }
};

template <int FIXED, bool PAIR>
__global__ __launch_bounds__(256) void qkv_pack_kernel(PackArgs pa) {
  const QkArgs& a = pa.qk;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.M) return;
  const bf16* base = a.x + (long)row * a.ldx;
  const PackStore ps{pa.table, pa.G, pa.R, pa.my_part, a.C / pa.G, (long)(pa.b_offset + row / a.rows_per_batch),
                     (long)(row % a.rows_per_batch), base + 2 * a.C};
  if (PAIR && a.rope && a.head_dim == 128) {  // the 1.3B shape: the pair path, as the in-place launcher takes
    qk_pair_row(a, row, lane, [&](int i, const float* yq, const float* yk) {
      ps.put<true>(i * 512 + lane * 8, yq);
      ps.put<false>(i * 512 + lane * 8, yk);
    });
    return;
  }
  bool rot = false;
  int fi = 0, hi_ = 0, wi = 0;
  if (a.rope) {
    const int t = a.tok_offset + row % a.rows_per_batch;
    if (t < a.F * a.H * a.W) {
      rot = true;
      fi = t / (a.H * a.W);
      hi_ = (t / a.W) % a.H;
      wi = t % a.W;
    }
  }
  rms_rope_one<FIXED>(base, a.wq, a, lane, fi, hi_, wi, rot, PackOne<true>{&ps});
  rms_rope_one<FIXED>(base + a.C, a.wk, a, lane, fi, hi_, wi, rot, PackOne<false>{&ps});
}

// The same LayerNorm with NW rows (one wave each) per workgroup sharing the per-batch modulation vectors
// (affine w / b, AdaLN scale / shift, gate) through LDS: staged once per workgroup instead of every wave
// reading up to 5 x C fp32 of them from L2 for its one row of C.  All NW rows lie in one batch row (the
// launcher checks rows_per_batch % NW == 0).  Per-element arithmetic as layernorm_mod_kernel, every multiply-add
// an explicit fma in both (so no contraction choice of the compiler's can tell them apart): bit-identical.
template <typename TI, typename TO, int FIXED, int NW>
__global__ __launch_bounds__(NW * 64) void layernorm_mod_shared_kernel(LnArgs a) {
  constexpr int C = FIXED * 512;
  __shared__ __attribute__((aligned(16))) float mod[5][C];
  const int row0 = blockIdx.x * NW;
  const long bo = (long)(row0 / a.rows_per_batch) * a.mod_bstride;
  const int row = row0 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  // this wave's row is loaded before the staging barrier, so the HBM reads of every wave are in flight while
  // the modulation vectors arrive from L2
  const bool live = row < a.M;
  const TI* x = (const TI*)a.x + (long)(live ? row : row0) * a.ldx;
  float v[FIXED][8];
#pragma unroll
  for (int i = 0; i < FIXED; ++i) load8<TI>(x + i * 512 + lane * 8, v[i]);
  for (int i = threadIdx.x; i < C / 4; i += NW * 64) {
    if (a.w) ((f32x4*)mod[0])[i] = ((const f32x4*)a.w)[i];
    if (a.b) ((f32x4*)mod[1])[i] = ((const f32x4*)a.b)[i];
    if (a.scale) {
      ((f32x4*)mod[2])[i] = ((const f32x4*)(a.scale + bo))[i];
      ((f32x4*)mod[3])[i] = ((const f32x4*)(a.shift + bo))[i];
    }
    if (a.gate) ((f32x4*)mod[4])[i] = ((const f32x4*)(a.gate + bo))[i];
  }
  __syncthreads();
  if (!live) return;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < FIXED; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[i][j];
  const float mean = wave_sum(s) / a.C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < FIXED; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; q = __builtin_fmaf(d, d, q); }
  const float rstd = rsqrtf(wave_sum(q) / a.C + a.eps);
  TO* out = (TO*)a.out + (long)row * a.ldo;
#pragma unroll
  for (int i = 0; i < FIXED; ++i) {
    const int c0 = i * 512 + lane * 8;
    float y[8], w8[8], b8[8], sc8[8], sh8[8], g8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = (v[i][j] - mean) * rstd;
    if (a.w) {
      load8<float>(mod[0] + c0, w8);
      if (a.b) load8<float>(mod[1] + c0, b8);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = __builtin_fmaf(y[j], w8[j], a.b ? b8[j] : 0.f);
    }
    if (a.scale) {
      load8<float>(mod[2] + c0, sc8);
      load8<float>(mod[3] + c0, sh8);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = __builtin_fmaf(y[j], 1.f + sc8[j], sh8[j]);
    }
    if (a.gate) {
      load8<float>(mod[4] + c0, g8);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = __builtin_fmaf(y[j], g8[j], v[i][j]);
    }
    store8<TO>(out + c0, y);
  }
}

// SA_LN_SHARED: 0 one wave per row reading the modulation from L2 (layernorm_mod_kernel); 8 / 16 rows per
// workgroup sharing it through LDS (read per call, for the A/B)
inline int ln_shared_rows() {
  const char* e = getenv("SA_LN_SHARED");
  return e ? atoi(e) : SA_LN_SHARED_DEFAULT;
}

template <typename TI, typename TO>
int launch_ln(const LnArgs& a, hipStream_t st) {
  const int nw = ln_shared_rows();
  const bool per_batch = a.scale || a.gate;  // batch-indexed vectors: a workgroup's rows must share the batch row
  if (a.C == 1536 && nw > 0 && (!per_batch || a.rows_per_batch % nw == 0) && (per_batch || a.w)) {
    if (nw == 16) {
      hipLaunchKernelGGL((layernorm_mod_shared_kernel<TI, TO, 3, 16>), dim3((a.M + 15) / 16), dim3(1024), 0, st, a);
      SA_LAUNCH_CHECK();
      return SA_OK;
    }
    if (nw == 8) {
      hipLaunchKernelGGL((layernorm_mod_shared_kernel<TI, TO, 3, 8>), dim3((a.M + 7) / 8), dim3(512), 0, st, a);
      SA_LAUNCH_CHECK();
      return SA_OK;
    }
  }
  if (a.C == 1536)
    hipLaunchKernelGGL((layernorm_mod_kernel<TI, TO, 3>), dim3((a.M + 3) / 4), dim3(256), 0, st, a);
  else if (a.C == 5120)
    hipLaunchKernelGGL((layernorm_mod_kernel<TI, TO, 10>), dim3((a.M + 3) / 4), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((layernorm_mod_kernel<TI, TO>), dim3((a.M + 3) / 4), dim3(256), 0, st, a);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

}  // namespace

// in_dtype / out_dtype: 0 = fp32, 1 = bf16
extern "C" int sa_layernorm_mod(const void* x, int64_t ldx, int in_dtype, void* out, int64_t ldo, int out_dtype,
                                const float* weight, const float* bias, const float* shift, const float* scale,
                                int64_t mod_bstride, const float* gate, int rows_per_batch, int M, int C, float eps,
                                void* stream) {
  if (!x || !out || M <= 0 || C <= 0 || C % 8 || C > 512 * MAXV || ldx % 8 || ldo % 8) return SA_ERR_ARG;
  if ((shift == nullptr) != (scale == nullptr)) return SA_ERR_ARG;
  if ((scale || gate) && rows_per_batch <= 0) return SA_ERR_ARG;
  if (gate && (out_dtype != 0 || !scale)) return SA_ERR_ARG;
  LnArgs a{x, ldx, out, ldo, weight, bias, shift, scale, mod_bstride, gate, rows_per_batch > 0 ? rows_per_batch : 1,
           M, C, eps};
  hipStream_t st = (hipStream_t)stream;
  if (in_dtype == 0 && out_dtype == 1) return launch_ln<float, bf16>(a, st);
  if (in_dtype == 0 && out_dtype == 0) return launch_ln<float, float>(a, st);
  if (in_dtype == 1 && out_dtype == 1) return launch_ln<bf16, bf16>(a, st);
  if (in_dtype == 1 && out_dtype == 0) return launch_ln<bf16, float>(a, st);
  return SA_ERR_ARG;
}

extern "C" int sa_qk_rmsnorm_rope(void* x, int64_t ldx, int q_col, int k_col, const float* wq, const float* wk, int M,
                                  int C, int head_dim, float eps, const float* rope, int rows_per_batch,
                                  int tok_offset, int F, int H, int W, int n_frame_pairs, int n_height_pairs,
                                  void* stream) {
  if (!x || !wq || M <= 0 || C <= 0 || C % 8 || C > 512 * MAXV || ldx % 8) return SA_ERR_ARG;
  if (k_col >= 0 && !wk) return SA_ERR_ARG;
  if (rope && (rows_per_batch <= 0 || head_dim % 8 || F <= 0 || H <= 0 || W <= 0)) return SA_ERR_ARG;
  QkArgs a{(bf16*)x, ldx, q_col, k_col, wq, wk, M, C, head_dim, eps, rope, rows_per_batch > 0 ? rows_per_batch : 1,
           tok_offset, F, H, W, n_frame_pairs, n_height_pairs};
  static const bool generic = getenv("SA_QK_GENERIC") != nullptr;  // A/B switch, read once
  if (rope && k_col >= 0 && C == 1536 && head_dim == 128 && !generic)
    hipLaunchKernelGGL(qk_rmsnorm_rope_pair_kernel, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, a);
  else if (C == 1536)
    hipLaunchKernelGGL(qk_rmsnorm_rope_kernel<3>, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, a);
  else if (C == 5120)
    hipLaunchKernelGGL(qk_rmsnorm_rope_kernel<10>, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(qk_rmsnorm_rope_kernel<0>, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, a);
  SA_LAUNCH_CHECK();
  return SA_OK;
}

extern "C" int sa_qkv_pack(const void* x, int64_t ldx, const float* wq, const float* wk, int M, int C, int head_dim,
                           float eps, const float* rope, int rows_per_batch, int tok_offset, int F, int H, int W,
                           int n_frame_pairs, int n_height_pairs, const int64_t* table, int G, int R, int my_part,
                           int b_offset, void* stream) {
  if (!x || !wq || !wk || !table || M <= 0 || C <= 0 || C % 512 || C > 512 * MAXV || ldx % 8 || ldx < 3 * C)
    return SA_ERR_ARG;
  if (G <= 0 || R <= 0 || my_part < 0 || my_part >= R || b_offset < 0 || rows_per_batch <= 0) return SA_ERR_ARG;
  if (C % G || (C / G) % 8) return SA_ERR_ARG;
  if (rope && (head_dim % 8 || F <= 0 || H <= 0 || W <= 0)) return SA_ERR_ARG;
  PackArgs pa{QkArgs{(bf16*)x, ldx, 0, C, wq, wk, M, C, head_dim, eps, rope, rows_per_batch, tok_offset, F, H, W,
                     n_frame_pairs, n_height_pairs},
              (const long*)table, G, R, my_part, b_offset};
  static const bool generic = getenv("SA_QK_GENERIC") != nullptr;  // the in-place launcher's A/B switch
  if (C == 1536 && !generic)
    hipLaunchKernelGGL((qkv_pack_kernel<3, true>), dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, pa);
  else if (C == 1536)
    hipLaunchKernelGGL((qkv_pack_kernel<3, false>), dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, pa);
  else if (C == 5120)
    hipLaunchKernelGGL((qkv_pack_kernel<10, false>), dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, pa);
  else
    hipLaunchKernelGGL((qkv_pack_kernel<0, false>), dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, pa);
  SA_LAUNCH_CHECK();
  return SA_OK;
}
