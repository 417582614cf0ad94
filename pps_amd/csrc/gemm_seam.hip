// The bottleneck seam: branch2c of block i and branch2a of block i+1 in one
// persistent kernel (ResNet.py:276-333 bottleneck_transformation: conv1x1
// 2c + AffineChannel + Sum(shortcut) + Relu, then the next block's conv1x1
// 2a + AffineChannel + Relu), for the identity-shortcut blocks of res2 / res3
// (K1 = 64 / 128 bottleneck channels, N1 = 4 K1 trunk channels).
//
// Unfused, the trunk T = relu(A W2c^T s + t + R) is written by 2c and read
// back whole by the next 2a: res2 moves 453 + 252 MB for 12.9 GFLOP at batch
// 64.  Here a workgroup owns 128 rows (16 per wave) and walks the trunk's
// columns in stages of CG: per stage each wave computes its 16 x CG block of
// 2c from its bf16x3 A fragments (split once per tile), finishes it (scale /
// shift, residual, ReLU -- the residual read and the T write as whole row
// segments through a wave-private LDS scratch), and feeds the finished block
// straight into 2a as the next CG / 32 K chunks of its accumulators, read
// back from the scratch in the MFMA operand layout.  T is still written (the
// residual of block i+1) but never read back: 503 MB instead of 705 MB.
//
// Weights: the stage's W2c rows [cg CG, +CG) x K1 and W2a columns
// [cg CG, +CG) x N2, bf16x3 planes, 48 KB, staged through registers into a
// double-buffered LDS slab shared by the 8 waves (one barrier per stage); the
// next stage's slab, residual block and (at stage 0) the next tile's A rows
// are requested before the current stage computes.
//
// Arithmetic: 2c = the six terms of mfma16_x3t per 32-wide K chunk in chunk
// order then fma(acc, scale, shift) + residual, ReLU; 2a the same on T's
// exact bf16x3 split with its K chunks in increasing order -- the sequence of
// the S = 16 tiles (38-55): both outputs equal the unfused layers' bits.
#include <cstdlib>

#include "gemm_x3_common.hpp"

namespace pps {


namespace {

template <int K1, int N1, int N2, int CG, int W>
struct SeamCfg {
  static constexpr int NW = W;                 // waves = 16-row blocks per tile
  static constexpr int ROWS = 16 * W;
  static constexpr int NCG = N1 / CG;          // stages per tile
  static constexpr int KC1 = K1 / 32;          // 2c K chunks
  static constexpr int JC = CG / 16;           // 2c column blocks per stage
  static constexpr int KC2 = CG / 32;          // 2a K chunks per stage
  static constexpr int JA = N2 / 16;           // 2a column blocks
  static constexpr int W2C = CG * K1 * 6;      // W2c slab bytes
  static constexpr int W2A = N2 * CG * 6;      // W2a slab bytes
  static constexpr int STAGE = W2C + W2A;
  static constexpr int PPT = STAGE / 16 / (64 * W);  // 16-B pieces per thread
  static constexpr int LDT = CG + 4;           // scratch row (floats)
  static constexpr int SCR = 16 * LDT * 4;     // scratch bytes per wave
  static constexpr int C4 = CG / 4;            // lanes per scratch row (row layout)
  static constexpr int RPI = 64 / C4;          // rows per row-layout instruction
  static constexpr int NIT = 16 / RPI;         // row-layout instructions per 16 rows
  static constexpr int SSH = (2 * N1 + 2 * N2) * 4;
  static constexpr int LDS = 2 * STAGE + W * SCR + SSH;
  // the next tile's A rows requested two stages ahead (K1 = 128: 32 more
  // live registers than the 256 of a two-wave-per-SIMD kernel allow)
  static constexpr bool PREA = K1 <= 64;
  // residual blocks requested PD stages ahead (an HBM-bound kernel needs
  // ~64 KB in flight per CU: two stages of 32 KB at CG = 64); PD = 2 runs
  // the NCG stages of a tile unrolled, the ring slot of a stage = its index
  static constexpr int PD = (K1 <= 64 && NCG <= 4) ? 2 : 1;
  static_assert(N1 % CG == 0 && CG % 32 == 0 && K1 % 32 == 0 && N2 % 16 == 0, "seam shape");
  static_assert(PPT * 16 * 64 * W == STAGE && PPT % 2 == 0 && W2C == W2A,
                "slab does not split into two equal halves of pieces");
  static_assert(RPI * C4 == 64 && NIT * RPI == 16, "scratch row layout");
  static_assert(N2 % CG == 0 && NCG % 2 == 0 && NCG >= 2, "2a epilogue in CG-column groups; stage pairs");
  static_assert(LDS <= 160 * 1024, "seam LDS");
};

template <int K1, int N1, int N2, int CG, int W>
__global__ void __launch_bounds__(64 * W)
seam_kernel(SeamParams p, int ntiles) {
  using C = SeamCfg<K1, N1, N2, CG, W>;
  constexpr int kSeamWaves = W;
  constexpr int kSeamRows = C::ROWS;
  __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, h = lane >> 4;
  const int bsw = sw64(r16);
  float* scr = reinterpret_cast<float*>(lds + 2 * C::STAGE) + wave * (C::SCR / 4);
  float* s_s2c = reinterpret_cast<float*>(lds + 2 * C::STAGE + kSeamWaves * C::SCR);
  float* s_t2c = s_s2c + N1;
  float* s_s2a = s_t2c + N1;
  float* s_t2a = s_s2a + N2;
  for (int c = threadIdx.x; c < N1; c += 64 * kSeamWaves) {
    s_s2c[c] = p.s2c[c];
    s_t2c[c] = p.t2c[c];
  }
  for (int c = threadIdx.x; c < N2; c += 64 * kSeamWaves) {
    s_s2a[c] = p.s2a[c];
    s_t2a[c] = p.t2a[c];
  }
  const rsrc_t ra = make_rsrc(p.a, (uint32_t)((int64_t)p.M * K1 * 4));
  const rsrc_t rr = make_rsrc(p.res, (uint32_t)((int64_t)p.M * N1 * 4));
  const rsrc_t rt = make_rsrc(p.t, (uint32_t)((int64_t)p.M * N1 * 4));
  const rsrc_t ry = make_rsrc(p.y, (uint32_t)((int64_t)p.M * N2 * 4));

  // ---- stage slab pieces of this thread: global element offset and LDS
  // byte offset of piece u (recomputed per use: a handful of integer ops
  // instead of 2 * PPT live registers); stage cg adds cg * CG to the W2c row
  // / W2a column
  auto piece = [&](int i, int cg, int& goff, int& loff) -> const uint16_t* {
    const int u = threadIdx.x + i * 64 * kSeamWaves;
    const int slot = u & 3;
    const int rest = u >> 2;
    if (u * 16 < C::W2C) {   // W2c: [kc][pl][n][32]
      const int n = rest % CG, pk = rest / CG, kc = pk / 3, pl = pk - 3 * kc;
      goff = pl * N1 * K1 + (cg * CG + n) * K1 + kc * 32 + slot * 8;
      loff = (pk * CG + n) * 64 + ((slot ^ sw64(n)) << 4);
      return p.w2c;
    }
    const int r2 = rest - C::W2C / 64;   // W2a: [kc2][pl][n][32]
    const int n = r2 % N2, pk = r2 / N2, kc = pk / 3, pl = pk - 3 * kc;
    goff = pl * N2 * N1 + n * N1 + cg * CG + kc * 32 + slot * 8;
    loff = C::W2C + (pk * N2 + n) * 64 + ((slot ^ sw64(n)) << 4);
    return p.w2a;
  };
  // the slab in two halves of PPT / 2 pieces: the W2c half (read by 2c) and
  // the W2a half (read by 2a), so the staging registers hold one half at a
  // time: the next stage's W2c half is requested at the top of a stage and
  // stored after 2c, its W2a half requested then and stored after 2a
  constexpr int HP = C::PPT / 2;
  auto wload = [&](int cg, int half, u32x4 (&wr)[HP]) {
#pragma unroll
    for (int i = 0; i < HP; ++i) {
      int g, l;
      const uint16_t* base = piece(half * HP + i, cg, g, l);
      wr[i] = *reinterpret_cast<const u32x4*>(base + g);
    }
  };
  auto wstore = [&](int buf, int half, const u32x4 (&wr)[HP]) {
#pragma unroll
    for (int i = 0; i < HP; ++i) {
      int g, l;
      (void)piece(half * HP + i, 0, g, l);
      *reinterpret_cast<u32x4*>(lds + buf * C::STAGE + l) = wr[i];
    }
  };
  // A rows of this wave: lane (r16, h) holds K [32 kc + 8 h, +8) of row r16
  auto aload = [&](int tile, f32x4 (&av)[C::KC1][2]) {
    const int m = tile * kSeamRows + wave * 16 + r16;
    const int o = (tile < ntiles && m < p.M) ? (m * K1 + 8 * h) * 4 : kOOB;
#pragma unroll
    for (int kc = 0; kc < C::KC1; ++kc) {
      av[kc][0] = bload(ra, o == kOOB ? kOOB : o + kc * 128);
      av[kc][1] = bload(ra, o == kOOB ? kOOB : o + kc * 128 + 16);
    }
  };
  // residual block of stage cg in row layout: lane -> row RPI it + lane / C4,
  // columns cg CG + 4 (lane % C4)
  auto rload = [&](int tile, int cg, f32x4 (&rv)[C::NIT]) {
#pragma unroll
    for (int it = 0; it < C::NIT; ++it) {
      const int m = tile * kSeamRows + wave * 16 + C::RPI * it + lane / C::C4;
      const int o = (tile < ntiles && m < p.M) ? (m * N1 + cg * CG + 4 * (lane % C::C4)) * 4 : kOOB;
      rv[it] = bload(rr, o);
    }
  };

  const int t0 = blockIdx.x;
  f32x4 av[C::KC1][2];
  f32x4 rv0[C::NIT], rv1[C::NIT];
  f32x4 rvr[C::PD == 2 ? C::NCG : 1][C::NIT];
  u32x4 wr[HP];
  aload(t0, av);
  rload(t0, 0, rv0);
  if constexpr (C::PD == 2) {
#pragma unroll
    for (int it = 0; it < C::NIT; ++it) rvr[0][it] = rv0[it];
    rload(t0, 1, rvr[1]);
  }
  wload(0, 0, wr);
  wstore(0, 0, wr);
  wload(0, 1, wr);
  wstore(0, 1, wr);
  __syncthreads();

  float amt = 0.f, amy = 0.f;  // max of the trunk / next-branch2a outputs (ReLU: >= 0)
  for (int tile = t0; tile < ntiles; tile += gridDim.x) {
    const int tnext = tile + gridDim.x;
    bf16x8 fa[C::KC1][3];
#pragma unroll
    for (int kc = 0; kc < C::KC1; ++kc) split8(av[kc][0], av[kc][1], fa[kc][0], fa[kc][1], fa[kc][2]);
    f32x4 acc2a[C::JA];
#pragma unroll
    for (int j = 0; j < C::JA; ++j) acc2a[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int mbase = tile * kSeamRows + wave * 16;
    // one stage: rcur = its residual block (requested a stage ago), rnxt
    // receives the next stage's
    auto stage = [&](int cg, f32x4 (&rcur)[C::NIT], f32x4 (&rnxt)[C::NIT], bool next_a,
                     int rl_tile, int rl_cg) {
      const int buf = cg & 1;   // NCG is even: stage parity repeats every tile
      // next stage's weights and residual (stage 0 of the next tile at the
      // end); the next tile's A rows two stages before they are split
      const bool last = cg + 1 == C::NCG;
      const int cgn = last ? 0 : cg + 1;
      wload(cgn, 0, wr);
      rload(rl_tile, rl_cg, rnxt);
      if (next_a) aload(tnext, av);
      const unsigned char* sl = lds + buf * C::STAGE;
      // 2c: this wave's 16 x CG block
      f32x4 acc[C::JC];
#pragma unroll
      for (int j = 0; j < C::JC; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < C::KC1; ++kc) {
#pragma unroll
        for (int j = 0; j < C::JC; ++j) {
          bf16x8 fb[3];
          const unsigned char* bp = sl + ((kc * 3) * CG + 16 * j + r16) * 64 + ((h ^ bsw) << 4);
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) fb[pl] = *reinterpret_cast<const bf16x8*>(bp + pl * CG * 64);
          acc[j] = mfma16_x3t(fa[kc], fb, acc[j]);
        }
        if (kc & 1) asm volatile("" ::: "memory");   // bounded read-ahead (registers)
      }
      // epilogue through the scratch: park, finish in row layout (residual,
      // T store), leave the finished block for the 2a fragments
#pragma unroll
      for (int j = 0; j < C::JC; ++j)
        *reinterpret_cast<f32x4*>(scr + r16 * C::LDT + 16 * j + 4 * h) = acc[j];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int it = 0; it < C::NIT; ++it) {
        const int row = C::RPI * it + lane / C::C4, col = 4 * (lane % C::C4);
        const f32x4 a4 = *reinterpret_cast<const f32x4*>(scr + row * C::LDT + col);
        const f32x4 s4 = *reinterpret_cast<const f32x4*>(s_s2c + cg * CG + col);
        const f32x4 t4 = *reinterpret_cast<const f32x4*>(s_t2c + cg * CG + col);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(__builtin_fmaf(a4[e], s4[e], t4[e]) + rcur[it][e], 0.f);
        const int m = mbase + row;
        const int o = m < p.M ? (m * N1 + cg * CG + col) * 4 : kOOB;
        if (m < p.M) amt = fmaxf(amt, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rt, o, 0, kStAux);
        *reinterpret_cast<f32x4*>(scr + row * C::LDT + col) = v;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wstore(buf ^ 1, 0, wr);
      wload(cgn, 1, wr);
      // 2a: the finished block as K chunks cg KC2 .. of the next layer
#pragma unroll
      for (int c = 0; c < C::KC2; ++c) {
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(scr + r16 * C::LDT + 32 * c + 8 * h);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(scr + r16 * C::LDT + 32 * c + 8 * h + 4);
        bf16x8 f2[3];
        split8(x0, x1, f2[0], f2[1], f2[2]);
#pragma unroll
        for (int j = 0; j < C::JA; ++j) {
          bf16x8 fb[3];
          const unsigned char* bp =
              sl + C::W2C + ((c * 3) * N2 + 16 * j + r16) * 64 + ((h ^ bsw) << 4);
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) fb[pl] = *reinterpret_cast<const bf16x8*>(bp + pl * N2 * 64);
          acc2a[j] = mfma16_x3t(f2, fb, acc2a[j]);
          // at most four blocks' weight fragments in flight (the compiler
          // would hoist all JA blocks' reads and spill)
          if ((j & 3) == 3) asm volatile("" ::: "memory");
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // scratch reads done
      wstore(buf ^ 1, 1, wr);
      __syncthreads();
    };
    // two stages per trip (the residual ring's buffers keep static names);
    // the last two stages outside the loop, where the next tile's A rows are
    // requested (a load inside the loop would keep them live all along)
    if constexpr (C::PD == 2) {
#pragma unroll
      for (int cg = 0; cg < C::NCG; ++cg) {
        const int nx = cg + 2;
        stage(cg, rvr[cg], rvr[nx % C::NCG], cg == C::NCG - 2, nx < C::NCG ? tile : tnext,
              nx % C::NCG);
      }
    } else {
      for (int cg = 0; cg < C::NCG - 2; cg += 2) {
        stage(cg, rv0, rv1, false, tile, cg + 1);
        stage(cg + 1, rv1, rv0, false, tile, cg + 2);
      }
      stage(C::NCG - 2, rv0, rv1, C::PREA, tile, C::NCG - 1);
      stage(C::NCG - 1, rv1, rv0, false, tnext, 0);
    }
    // 2a epilogue in CG-column groups through the scratch: Y = relu(acc s + t)
#pragma unroll
    for (int g = 0; g < N2 / CG; ++g) {
#pragma unroll
      for (int j = 0; j < C::JC; ++j)
        *reinterpret_cast<f32x4*>(scr + r16 * C::LDT + 16 * j + 4 * h) = acc2a[g * C::JC + j];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int it = 0; it < C::NIT; ++it) {
        const int row = C::RPI * it + lane / C::C4, col = 4 * (lane % C::C4);
        const f32x4 a4 = *reinterpret_cast<const f32x4*>(scr + row * C::LDT + col);
        const f32x4 s4 = *reinterpret_cast<const f32x4*>(s_s2a + g * CG + col);
        const f32x4 t4 = *reinterpret_cast<const f32x4*>(s_t2a + g * CG + col);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(__builtin_fmaf(a4[e], s4[e], t4[e]), 0.f);
        const int m = mbase + row;
        const int o = m < p.M ? (m * N2 + g * CG + col) * 4 : kOOB;
        if (m < p.M) amy = fmaxf(amy, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ry, o, 0, kStAux);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (!C::PREA) aload(tnext, av);   // (res3: requested earlier it would spill)
  }
  if (p.amax_t) amax_commit(p.amax_t, amt);
  if (p.amax_y) amax_commit(p.amax_y, amy);
}

template <int K1, int N1, int N2, int CG, int W>
int launch_seam(const SeamParams& p, hipStream_t st) {
  constexpr int kSeamRows = 16 * W;
  const int ntiles = (p.M + kSeamRows - 1) / kSeamRows;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = ntiles < cus ? ntiles : cus;
  hipLaunchKernelGGL((seam_kernel<K1, N1, N2, CG, W>), dim3((unsigned)grid), dim3(64 * W), 0, st,
                     p, ntiles);
  PPS_CHECK_LAUNCH("seam_kernel");
  return PPS_OK;
}

}  // namespace

bool seam_supported(int K1, int N1, int N2) {
  return (K1 == 64 && N1 == 256 && N2 == 64) || (K1 == 128 && N1 == 512 && N2 == 128);
}

int launch_seam_x3(const SeamParams& p, int K1, int N1, int N2, hipStream_t st) {
  if (p.M <= 0) return PPS_OK;
  // res2 (M = 196,608 at batch 64): 128-row tiles, 6 per CU; res3 (M =
  // 49,152): 128-row tiles leave half the CUs one tile behind (384 tiles);
  // 96-row tiles (6 waves) spill
  if (K1 == 64 && N1 == 256 && N2 == 64) return launch_seam<64, 256, 64, 64, 8>(p, st);
  if (K1 == 128 && N1 == 512 && N2 == 128) {
    // PPS_SEAM_W3 (probes): 4 = 64-row tiles, one wave per SIMD, 3 per CU
    static const int w3 = [] {
      const char* e = getenv("PPS_SEAM_W3");
      return e ? atoi(e) : 8;
    }();
    if (w3 == 4) return launch_seam<128, 512, 128, 32, 4>(p, st);
    return launch_seam<128, 512, 128, 32, 8>(p, st);
  }
  set_error("bottleneck seam: shapes (K1, N1, N2) = (64, 256, 64) or (128, 512, 128) only");
  return PPS_ERR_INVALID_ARG;
}

}  // namespace pps
