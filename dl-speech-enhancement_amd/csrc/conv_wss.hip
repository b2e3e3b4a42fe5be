// Sample-tile warp-specialised conv (k_conv_wss): the conv primitive of
// conv.hip (include/sel.h sel_conv_fwd) for short sequences, T <= 400 — the
// C3 generator's 256-wide stage: the RU256 k7 convs and their adjoints
// (models/autoencoder/modules/residual_unit.py:43-46 over
// layers/conv_layer.py:139-142), the stride-5 down conv in its phase-packed
// 3-tap form and the 2-tap transposed conv (conv_layer.py:180-183).
//
// Why a second warp-specialised kernel.  k_conv_ws_bf16 computes 256 x 128
// tiles: a 400-row sample takes two row tiles, the second 56% useful, so the
// chip computes 1.28x the outputs, one tile per CU, 8 waves of 64 x 64.
// Here one tile is a WHOLE sample x 64 output channels (B x N/64 tiles: 256 at
// C3), so no output row is computed twice or padded beyond the 16-row MFMA
// strip (400 = 25 strips of 16), and the 25 strips are dealt so every SIMD gets
// the same MFMA count:
//   - 4 consumer waves (one per SIMD) on v_mfma_f32_16x16x32_bf16; wave w owns
//     Q = S/4 full strips (all 4 column strips: 4Q accumulators) plus R = S%4
//     (strip, column-strip) pairs of the last S%4 strips: 4Q + R MFMAs per
//     (tap, 32-channel chunk) on every SIMD (25 at S = 25);
//   - per tap a wave reads 4 + 1 weight fragments and Q + R input fragments
//     (ds_read_b128) for 4Q + R MFMAs (0.48 reads per 16-cycle MFMA at S = 25);
//   - 4 producer waves DMA each 32-channel chunk (the input span of T + halo
//     rows and the KT x 64 weight rows, 64-B LDS rows, global_load_lds_dwordx4
//     1-KB pieces) into a 2-slot ring one chunk ahead and apply the input ELU
//     in place (each lane rewrites the 16 B its own DMA landed).
// LDS rows are 64 B: 16-B slot p of row r holds source slot p ^ wss_swz(r), so
// the 16 lanes of each ds_read_b128 lane group hit 16 distinct 16-B bank groups
// (the DMA destination is lane-linear: the swizzle is applied to the source).
// Epilogue: accumulators -> fp32 [T][64 + 4] tile over the drained ring, then
// all 8 waves write 16-B row-contiguous output vectors with the bias, ELU'(aux)
// and residual terms of the conv.hip epilogue (same order, same roundings).
// The MFMA shape differs from k_conv_ws_bf16's 32x32x16, so the fp32 sums are
// ordered differently: outputs agree to bf16 rounding, not bit for bit
// (tests/test_gpu_c3.py checks every variant against fp64 of the same operands).
#include "conv_common.h"

namespace sel {
namespace conv {

constexpr int WSS_CK = 32;                 // channels per chunk = one MFMA k-step
constexpr int WSS_ROWB = WSS_CK * 2;       // bytes per LDS row
constexpr int WSS_RPP = 1024 / WSS_ROWB;   // LDS rows per 1-KB DMA piece
constexpr int WSS_CMAX = 4096;             // input channels the zero source covers
constexpr int WSS_NB = 2;                  // ring slots

__device__ __attribute__((aligned(64))) __bf16 g_wss_zero[WSS_CMAX];

// KT taps, S 16-row strips per tile, BN output channels per tile (64 or 128:
// NCS = BN / 16 column strips).  Wave w owns Q = S / 4 full strips (all NCS
// column strips) plus E of the R * NCS (strip, column strip) pairs of the last
// R = S % 4 strips.  SPT > 1 (round 6): a tile is SPT whole short samples (T =
// 16 S / SPT rows each: the C3 T = 80 convs, five samples per 400-row tile),
// each staged as its own segment of T + halo rows (rounded to 16) so a strip
// never reads another sample's rows.
template <int KT, int S, int BN, int SPT = 1>
struct WssGeo {
  static constexpr int Q = S / 4, R = S % 4, NCS = BN / 16, E = R * NCS / 4;
  static_assert((R * NCS) % 4 == 0, "extra pairs split evenly over the four consumers");
  static constexpr int EP = BN + 4;  // fp32 epilogue tile pitch
  static constexpr int XROWS = SPT == 1 ? (S * 16 + F4_HALOMAX + WSS_RPP - 1) / WSS_RPP * WSS_RPP  // staged input rows
                                        : S * 16 + SPT * F4_HALOMAX;
  static constexpr int XI = XROWS / WSS_RPP;            // input DMA pieces per chunk
  static constexpr int WI = KT * BN / WSS_RPP;          // weight DMA pieces per chunk
  static constexpr int TI = XI + WI;
  static constexpr int PW = (TI + 3) / 4;               // pieces per producer wave
  static constexpr int SLOT = (XROWS + KT * BN) * WSS_ROWB;
  static constexpr int RING = WSS_NB * SLOT;
  static constexpr int EPI = S * 16 * EP * 4;
  // the ELU pass reads eight pieces 4 KB apart per group (k_conv_wss)
  static constexpr int PX = (XI + 3) / 4, NGRP = (PX + 7) / 8;
  static constexpr int ELUR = (WSS_NB - 1) * SLOT + (4 * (8 * NGRP - 1) + 3 + 1) * 1024;
  static constexpr int LDS0 = RING > EPI ? RING : EPI;
  static constexpr int LDS = LDS0 > ELUR ? LDS0 : ELUR;
};

// 16-B slot XOR of LDS row `row`: ds_read_b128 serves a wave in four 16-lane
// groups {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} (+32); a fragment read puts
// lanes l on rows r0 + (l & 15), slot l >> 4, so each group holds rows r0 + j
// for every j mod 16, in slots that differ by bit 0.  With (row >> 1) & 2 the
// 16 lanes of every group hit 16 distinct 16-B bank groups for ANY r0 (the taps
// shift r0 by k * dil), brute-force checked; (row >> 2) & 3 left them 2-way
// (PMC: SQ_LDS_BANK_CONFLICT 44% of SQ_LDS_IDX_ACTIVE).
__device__ __forceinline__ int wss_swz(int row) { return (row >> 1) & 2; }

// RU (round 6, the 128-channel residual unit's forward, residual_unit.py:43-46,
// on the (16, 128) tile): `out` receives h = conv_k7(ELU(x)) + b1, `out2` the
// unit's output x + W2 ELU(h) + b2 (`res` = x).  LDS after the main loop:
//   - W2 (128 x 128 bf16, 16-B slot p of row n at p ^ (n & 15)) and b1, DMA'd /
//     written by the producers once the ring's slot 0 is free (after the
//     second-to-last chunk), so they are in place when the consumers finish;
//   - the consumers add b1 to their accumulators and write h as bf16 rows
//     [256][136] (no fp32 tile); all waves store h row-contiguous and ELU it in
//     place (each 16-B vector by its own thread);
//   - wave w: rows 32w .. + 31 x 128 channels, 32x32x16 MFMAs in k_pw_bf16's
//     operand and channel order; fp32 tile; + b2, + x (k_pw_bf16's epilogue).
// Bit-identical to k_conv_wss + k_pw_bf16 (tests/test_gpu_conv.py).
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
constexpr int WSS_PWP = 128 + 8;           // bf16 pitch of the h rows (conflict-free b128 reads)
constexpr int WSS_B1_OFF = 128 * 128 * 2;  // byte offsets: W2 at 0, b1, the h rows
constexpr int WSS_HS_OFF = WSS_B1_OFF + 128 * 4;

template <int KT, int S, int BN, typename TO, int SPT = 1, bool RU = false>
__global__ __launch_bounds__(512) void k_conv_wss(Args a, const __bf16* __restrict__ in,
                                                  const __bf16* __restrict__ wp, const float* __restrict__ bias,
                                                  const TO* __restrict__ aux, const TO* __restrict__ res,
                                                  TO* __restrict__ out, int ncol, int tm, int dbg,
                                                  const __bf16* __restrict__ w2, const float* __restrict__ b2,
                                                  TO* __restrict__ out2) {
  using G = WssGeo<KT, S, BN, SPT>;
  static_assert(!RU || (BN == 128 && S == 16 && SPT == 1 && sizeof(TO) == 2), "RU: the (16, 128) bf16 tile");
  static_assert(!RU || (WSS_HS_OFF + S * 16 * WSS_PWP * 2 <= G::SLOT + G::SLOT && G::SLOT >= WSS_B1_OFF + 512 &&
                        G::EPI <= G::LDS), "RU LDS layout: W2 and b1 inside ring slot 0");
  constexpr int Q = G::Q, NCS = G::NCS, E = G::E, XR = G::XROWS, XI = G::XI, TI = G::TI, PW = G::PW;
  constexpr int EP = G::EP;
  static_assert(2 * PW < 64, "vmcnt range");
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // tile = tm rows of one sample (tm <= 16 S; T = 400: the whole sample) x 64
  // output channels
  int64_t mt;
  int nt;
  xcd_tile(ncol, mt, nt);
  const int T = a.T;
  const int64_t nsamp = a.rows / T;
  // SPT == 1: tile = tm rows of sample b from row t0; SPT > 1: samples
  // b .. b + SPT - 1 whole (the last tile may hold fewer), their rows contiguous
  const int tps = SPT == 1 ? (T + tm - 1) / tm : 1;
  const int64_t b = SPT == 1 ? mt / tps : mt * SPT;
  const int t0 = SPT == 1 ? int(mt - b * tps) * tm : 0;
  const int nsp = SPT == 1 ? 1 : int(nsamp - b < SPT ? nsamp - b : SPT);  // samples in this tile
  const int mrows = SPT == 1 ? (T - t0 < tm ? T - t0 : tm) : nsp * T;
  const int64_t m0 = b * T + t0;
  const int n0 = nt * BN;
  const int nchunk = a.C / WSS_CK;
  const int span = SPT == 1 ? tm + (KT - 1) * a.dil : 0;
  // SPT > 1: each sample's segment is seg rows (T + halo, 16-row multiple)
  const int seg = SPT == 1 ? 0 : (T + (KT - 1) * a.dil + 15) / 16 * 16;
  // diagnostic (tune key 48 bit 4): s_memtime stamps of block phases, written
  // over the first output bytes at the end (st[0] start, [1] first chunk ready,
  // [2] consumer loop done, [3] tile in LDS, [4] end, [5]/[6] realtime start/end)
  uint64_t st[5] = {0, 0, 0, 0, 0};
  uint64_t rt0 = 0;
  if (dbg & 16) {
    st[0] = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }

  // epilogue operands: thread t owns the 16-B output vectors v = t + 512 u; their
  // ELU'(aux) and residual rows are requested early (producers after their
  // last DMA, consumers right after their MFMAs) so the epilogue does not wait
  // on HBM
  struct alignas(16) V8 { TO v[8]; };
  constexpr int NT = 512, VPR = BN / 8, EV = (S * 16 * VPR + NT - 1) / NT;  // VPR: 16-B vectors per row
  const int nvec = mrows * VPR;
  V8 av[EV], rv[EV];
  auto prefetch_epi = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < EV; ++u) {
      const int v = tid + u * NT;
      if (v >= nvec) break;
      const int64_t o = (m0 + v / VPR) * a.N + n0 + (v % VPR) * 8;
      if (aux) av[u] = *reinterpret_cast<const V8*>(aux + o);
      if (res) rv[u] = *reinterpret_cast<const V8*>(res + o);
    }
  };

  if (wave >= 4) {
    // ---------------- producers ----------------
    const int pw = wave - 4;
    // RU: b1 value of channel 64 pw + lane (pw < 2), staged with W2
    const float b1v = RU && pw < 2 && bias && a.bias_period ? bias[pw * 64 + lane] : 0.f;
    const __bf16* src[PW];
#pragma unroll
    for (int u = 0; u < PW; ++u) {
      const int q = u * 4 + pw < TI ? u * 4 + pw : TI - 1;  // a wave short of PW repeats the last piece
      const int rr = (q < XI ? q : q - XI) * WSS_RPP + (lane >> 2);
      const int ls = (lane & 3) ^ wss_swz(rr);
      if (q < XI) {
        int64_t bs = b;
        int rl = rr;
        bool inseg = rr < span;
        if constexpr (SPT > 1) {  // segment j = sample b + j: rows - pad .. of it
          const int j = rr / seg;
          rl = rr - j * seg;
          bs = b + j;
          inseg = j < nsp && rl < T + (KT - 1) * a.dil;
        }
        int ti = t0 + rl - a.pad;
        const bool valid = inseg && ((ti >= 0 && ti < T) || a.pad_mode == SEL_PAD_REPLICATE);
        ti = ti < 0 ? 0 : (ti >= T ? T - 1 : ti);
        src[u] = valid ? in + (bs * T + ti) * a.C + 8 * ls : g_wss_zero + 8 * ls;
      } else {
        const int k = rr / BN, n = rr % BN;
        src[u] = wp + (int64_t(n0 + n) * KT + k) * a.C + 8 * ls;
      }
    }
    const int xi_used = SPT == 1 ? (span + WSS_RPP - 1) / WSS_RPP   // input pieces holding rows < span
                                 : (nsp * seg + WSS_RPP - 1) / WSS_RPP;
    auto issue = [&](int ch) __attribute__((always_inline)) {
      unsigned char* const base = smem + (ch % WSS_NB) * G::SLOT;
#pragma unroll
      for (int u = 0; u < PW; ++u) {
        const int q = u * 4 + pw < TI ? u * 4 + pw : TI - 1;
        const int off = q < XI ? q * 1024 : XR * WSS_ROWB + (q - XI) * 1024;
        if (q >= xi_used && q < XI) continue;  // rows past the span: never read
        if (dbg & 2) continue;  // diagnostic (tune key 48 bit 1): no DMA
        __builtin_amdgcn_global_load_lds((const void*)(src[u] + ch * WSS_CK), (lds_ptr_t)(base + off), 16, 0, 0);
      }
    };
    // in-place ELU of this wave's input pieces (q = 4u + pw): the eight reads
    // and their wait in ONE asm statement (reads past the input pieces land in
    // the weight slices and are not written back), then ELU + write back.
    // Inline asm: a plain LDS access here would make hipcc drain vmcnt (the next
    // chunk's DMA) first; one statement: the compiler cannot hoist a use of a
    // result above the wait.
    constexpr int PX = G::PX, NGRP = G::NGRP;
    // (the reads past the input pieces stay inside the allocation; never written)
    static_assert(G::ELUR <= G::LDS, "ELU pass reads");
    auto elu_pass = [&](int ch) __attribute__((always_inline)) {
#pragma unroll
      for (int gq = 0; gq < NGRP; ++gq) {
        unsigned char* const base = smem + (ch % WSS_NB) * G::SLOT + lane * 16 + (pw + 32 * gq) * 1024;
        const unsigned addr = unsigned(reinterpret_cast<uintptr_t>(base));
        bf16x8 v[8];
        asm volatile(
            "ds_read_b128 %0, %8\n\t"
            "ds_read_b128 %1, %8 offset:4096\n\t"
            "ds_read_b128 %2, %8 offset:8192\n\t"
            "ds_read_b128 %3, %8 offset:12288\n\t"
            "ds_read_b128 %4, %8 offset:16384\n\t"
            "ds_read_b128 %5, %8 offset:20480\n\t"
            "ds_read_b128 %6, %8 offset:24576\n\t"
            "ds_read_b128 %7, %8 offset:28672\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
            : "v"(addr)
            : "memory");
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int q = (8 * gq + u) * 4 + pw;
          if (q >= XI || q >= xi_used) break;
          const bf16x8 e = __builtin_bit_cast(bf16x8, elu8(__builtin_bit_cast(uint4, v[u])));
          asm volatile("ds_write_b128 %0, %1 offset:%2" : : "v"(addr), "v"(e), "i"(u * 4096) : "memory");
        }
      }
    };
    // prologue: chunk 0 alone first (every CU bursts at once: one chunk lands
    // in about half the time of two), chunk 1 behind it, over chunk 0's ELU
    issue(0);
    ws_wait_vm<0>();
    if (nchunk > 1) issue(1);
    if (a.in_elu && !(dbg & 4)) elu_pass(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int ch = 0; ch < nchunk; ++ch) {
      // the consumers compute chunk ch; chunk ch + 1 (the only DMA in flight) lands, then its ELU
      if (ch + 1 < nchunk) {
        ws_wait_vm<0>();
        if (ch + 2 == nchunk) prefetch_epi();  // the last DMA has landed
        if (a.in_elu && !(dbg & 4)) elu_pass(ch + 1);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      // slot ch % 2 is free now
      if (ch + 2 < nchunk) issue(ch + 2);
      if constexpr (RU) {
        if (ch + 2 == nchunk) {  // slot 0 (nchunk even): W2 and b1 for the epilogue
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int j = u * 4 + pw, n = 4 * j + (lane >> 4), sl = (lane & 15) ^ (n & 15);
            __builtin_amdgcn_global_load_lds((const void*)(w2 + n * 128 + sl * 8), (lds_ptr_t)(smem + j * 1024), 16,
                                             0, 0);
          }
          if (pw < 2) reinterpret_cast<float*>(smem + WSS_B1_OFF)[pw * 64 + lane] = b1v;
        }
      }
    }
    if constexpr (RU) ws_wait_vm<0>();  // W2 has landed before the epilogue's first barrier
  } else {
    // ---------------- consumers ----------------
    const int w = wave;
    const int l16 = lane & 15, kq = lane >> 4;
    // lane's byte offset within a 16-row group of weight rows (row = 16 cs + l16
    // of tap k's BN rows; the swizzle depends on l16 only) and the extra pairs
    const int lane_w = l16 * WSS_ROWB + ((kq ^ wss_swz(l16)) << 4);
    constexpr int E1 = E > 0 ? E : 1;
    int xstrip[E1], xcol[E1];
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const int p = w * E + i;
      xstrip[i] = 4 * Q + p / NCS;
      xcol[i] = p % NCS;
    }
    // byte offset of strip st's first staged row (SPT > 1: its sample's segment;
    // a 16-row multiple, so the row swizzle of the tap reads is unchanged)
    const int sps = SPT == 1 ? S : T / 16;  // strips per sample
    auto sbase = [&](int st) { return SPT == 1 ? st * 1024 : ((st / sps) * seg + (st % sps) * 16) * WSS_ROWB; };
    int soff[Q > 0 ? Q : 1], xoff[E1];
#pragma unroll
    for (int i = 0; i < Q; ++i) soff[i] = sbase(w * Q + i);
#pragma unroll
    for (int i = 0; i < E; ++i) xoff[i] = sbase(xstrip[i]);
    floatx4 acc[Q][NCS], accx[E1];
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int c = 0; c < NCS; ++c) acc[i][c] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < E; ++i) accx[i] = floatx4{0.f, 0.f, 0.f, 0.f};

    bf16x8 fw[2][NCS], fx[2][Q], fwx[2][E1], fxx[2][E1];
    // fragments of tap k of the chunk in ring slot sl into buffer q
    static_assert(WSS_NB == 2, "two chunks per trip, one per ring slot");
    auto fetch = [&](int sl, int k, int q) __attribute__((always_inline)) {
      const unsigned char* const xb = smem + sl * G::SLOT;
      const unsigned char* const wb = xb + XR * WSS_ROWB;
#pragma unroll
      for (int c = 0; c < NCS; ++c)
        fw[q][c] = *reinterpret_cast<const bf16x8*>(wb + (k * BN + c * 16) * WSS_ROWB + lane_w);
      const int r = l16 + k * a.dil;  // + 16 s: the swizzle of row r + 16 s is r's
      int lx = r * WSS_ROWB + ((kq ^ wss_swz(r)) << 4);
      // computed here, per fetch (a few VALU): hoisted out of the loop, the
      // 2 x KT per-step addresses would take the registers the pipeline needs
      asm volatile("" : "+v"(lx));
#pragma unroll
      for (int i = 0; i < Q; ++i) fx[q][i] = *reinterpret_cast<const bf16x8*>(xb + soff[i] + lx);
#pragma unroll
      for (int i = 0; i < E; ++i) {
        fwx[q][i] = *reinterpret_cast<const bf16x8*>(wb + (k * BN + xcol[i] * 16) * WSS_ROWB + lane_w);
        fxx[q][i] = *reinterpret_cast<const bf16x8*>(xb + xoff[i] + lx);
      }
    };
    auto mfmas = [&](int q) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < Q; ++i)
#pragma unroll
        for (int c = 0; c < NCS; ++c)
          acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[q][c], fx[q][i], acc[i][c], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < E; ++i)
        accx[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fwx[q][i], fxx[q][i], accx[i], 0, 0, 0);
    };

    __syncthreads();
    if (dbg & 16) st[1] = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_setprio(2);
    if (dbg & 1) {  // diagnostic (tune key 48 bit 0): consumers skip the MFMA phase
      for (int ch = 0; ch < nchunk; ++ch) __builtin_amdgcn_s_barrier();
    } else {
      // one software pipeline over the (chunk, tap) steps, two chunks per trip so
      // the fragment buffer of every step is a compile-time index: step (ch, k)
      // issues the reads of the next step before its own MFMAs.  At a chunk's
      // last tap the wave's reads of that chunk are all done, so it meets the
      // producers' barrier there (slot ch free for chunk ch + 2, chunk ch + 1
      // ready) and the first reads of chunk ch + 1 overlap the last tap's MFMAs.
      fetch(0, 0, 0);
      for (int ch = 0; ch < nchunk; ch += 2) {
#pragma unroll
        for (int i = 0; i < 2 * KT; ++i) {
          // chunk ch + i / KT (ch even) sits in ring slot i / KT
          const int sl = i / KT, k = i % KT, q = i & 1;
          if (k + 1 < KT) {
            fetch(sl, k + 1, q ^ 1);
          } else {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            fetch(sl ^ 1, 0, q ^ 1);  // (after the last chunk: a dead read of the other slot, no branch)
          }
          mfmas(q);
          // the next step's reads go out between this step's MFMAs (one per
          // two), not as a burst that leaves the matrix pipe idle
          constexpr int NRD = NCS + Q + 2 * E, NMF = NCS * Q + E;
          constexpr int REST = NMF > 2 * NRD ? NMF - 2 * NRD : 0;
#pragma unroll
          for (int j = 0; j < NRD; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one DS read
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // two MFMAs
          }
          if (REST > 0) __builtin_amdgcn_sched_group_barrier(0x008, REST, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (dbg & 16) st[2] = __builtin_amdgcn_s_memtime();
    prefetch_epi();
    if constexpr (RU) {
      // h = acc + b1 (the fp32 epilogue's add) -> bf16 rows: lane -> time row
      // 16 s + l16, channels 16 c + 4 kq .. + 3 (E = 0 at S = 16)
      __bf16* const hs = reinterpret_cast<__bf16*>(smem + WSS_HS_OFF);
      const float* const b1s = reinterpret_cast<const float*>(smem + WSS_B1_OFF);
      const bool hb = bias && a.bias_period;
#pragma unroll
      for (int c = 0; c < NCS; ++c) {
        const floatx4 bb = *reinterpret_cast<const floatx4*>(b1s + c * 16 + 4 * kq);
#pragma unroll
        for (int i = 0; i < Q; ++i) {
          bf16x4 hv;
#pragma unroll
          for (int e = 0; e < 4; ++e) hv[e] = __bf16(hb ? acc[i][c][e] + bb[e] : acc[i][c][e]);
          *reinterpret_cast<bf16x4*>(hs + ((w * Q + i) * 16 + l16) * WSS_PWP + c * 16 + 4 * kq) = hv;
        }
      }
    } else {
      // accumulators -> fp32 [S*16][BN + 4] tile over the drained ring: lane ->
      // time row 16 s + l16, channels 16 c + 4 kq .. + 3
      float* const tile = reinterpret_cast<float*>(smem);
#pragma unroll
      for (int i = 0; i < Q; ++i)
#pragma unroll
        for (int c = 0; c < NCS; ++c)
          *reinterpret_cast<floatx4*>(tile + ((w * Q + i) * 16 + l16) * EP + c * 16 + 4 * kq) = acc[i][c];
#pragma unroll
      for (int i = 0; i < E; ++i)
        *reinterpret_cast<floatx4*>(tile + (xstrip[i] * 16 + l16) * EP + xcol[i] * 16 + 4 * kq) = accx[i];
    }
  }
  // (a raw barrier: __syncthreads() would also wait for the prefetched rows)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (dbg & 16) st[3] = __builtin_amdgcn_s_memtime();

  // epilogue by all 8 waves: 8 consecutive channels per thread, row-contiguous
  // 16-B accesses (aux / res fetched for every vector first); k_conv_ws_bf16's
  // term order
  const float* const tile = reinterpret_cast<const float*>(smem);
  if constexpr (RU) {
    __bf16* const hs = reinterpret_cast<__bf16*>(smem + WSS_HS_OFF);
    const __bf16* const ws = reinterpret_cast<const __bf16*>(smem);
    // h rows -> `out` (16-B row-contiguous), then ELU(h) in place for the 1x1
#pragma unroll
    for (int u = 0; u < EV; ++u) {
      const int v = tid + u * NT;
      if (v >= nvec) break;
      uint4* const p = reinterpret_cast<uint4*>(hs + (v / VPR) * WSS_PWP + (v % VPR) * 8);
      const uint4 hv = *p;
      *reinterpret_cast<uint4*>(out + (m0 + v / VPR) * a.N + (v % VPR) * 8) = hv;
      *p = elu8(hv);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // wave w: rows 32w .. 32w + 31 x all 128 output channels (4 32x32 blocks);
    // k_pw_bf16's fragments: weights first, channel groups g = 0 .. 7 in order
    const __bf16* const xb = hs + (wave * 32 + (lane & 31)) * WSS_PWP + 8 * (lane >> 5);
    bf16x8 xf[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) xf[g] = *reinterpret_cast<const bf16x8*>(xb + 16 * g);
    floatx16 acc2[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int n = cb * 32 + (lane & 31);
      bf16x8 wf[8];
#pragma unroll
      for (int g = 0; g < 8; ++g)
        wf[g] = *reinterpret_cast<const bf16x8*>(ws + n * 128 + (((2 * g + (lane >> 5)) ^ (n & 15)) * 8));
#pragma unroll
      for (int e = 0; e < 16; ++e) acc2[cb][e] = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) acc2[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[g], xf[g], acc2[cb], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's LDS reads are done: the fp32 tile goes over them
    float* const ot = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<floatx4*>(ot + (wave * 32 + (lane & 31)) * EP + cb * 32 + 8 * q + 4 * (lane >> 5)) =
            floatx4{acc2[cb][4 * q], acc2[cb][4 * q + 1], acc2[cb][4 * q + 2], acc2[cb][4 * q + 3]};
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // k_pw_bf16's epilogue: + b2, then + x (__fadd_rn), bf16
#pragma unroll
    for (int u = 0; u < EV; ++u) {
      const int v = tid + u * NT;
      if (v >= nvec) break;
      const int row = v / VPR, c8 = (v % VPR) * 8;
      const floatx4 lo = *reinterpret_cast<const floatx4*>(ot + row * EP + c8);
      const floatx4 hi = *reinterpret_cast<const floatx4*>(ot + row * EP + c8 + 4);
      float x[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (b2) {
        const floatx4 c0 = *reinterpret_cast<const floatx4*>(b2 + c8), c1 = *reinterpret_cast<const floatx4*>(b2 + c8 + 4);
        x[0] += c0[0], x[1] += c0[1], x[2] += c0[2], x[3] += c0[3];
        x[4] += c1[0], x[5] += c1[1], x[6] += c1[2], x[7] += c1[3];
      }
      V8 ov;
#pragma unroll
      for (int e = 0; e < 8; ++e) ov.v[e] = from_f<TO>(__fadd_rn(x[e], to_f(rv[u].v[e])));
      *reinterpret_cast<V8*>(out2 + (m0 + row) * a.N + c8) = ov;
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < EV; ++u) {
    const int v = tid + u * NT;
    if (v >= nvec) break;
    const int row = v / VPR, c8 = (v % VPR) * 8;
    const int64_t o = (m0 + row) * a.N + n0 + c8;
    const floatx4 lo = *reinterpret_cast<const floatx4*>(tile + row * EP + c8);
    const floatx4 hi = *reinterpret_cast<const floatx4*>(tile + row * EP + c8 + 4);
    float x[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    if (bias && a.bias_period) {
      if (a.bias_period % 8 == 0) {
        const float* const bp = bias + (n0 + c8) % a.bias_period;
        const floatx4 b0 = *reinterpret_cast<const floatx4*>(bp), b1 = *reinterpret_cast<const floatx4*>(bp + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] += b0[e], x[e + 4] += b1[e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] += bias[(n0 + c8 + e) % a.bias_period];
      }
    }
    if (aux) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] *= elu_grad_fast(to_f(av[u].v[e]));
    }
    if (res) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] += to_f(rv[u].v[e]);
    }
    V8 ov;
#pragma unroll
    for (int e = 0; e < 8; ++e) ov.v[e] = from_f<TO>(x[e]);
    if (!(dbg & 8)) *reinterpret_cast<V8*>(out + o) = ov;  // bit 3: diagnostic without the stores
  }
  if (dbg & 16) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (lane == 0) reinterpret_cast<uint64_t*>(out)[int64_t(blockIdx.x) * 16 + 8 + wave] = st[0];  // each wave's start
    if (tid == 0) {
      uint64_t* const d = reinterpret_cast<uint64_t*>(out) + int64_t(blockIdx.x) * 16;
      d[0] = st[0];
      d[1] = st[1];
      d[2] = st[2];
      d[3] = st[3];
      d[4] = __builtin_amdgcn_s_memtime();
      d[5] = rt0;
      d[6] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// Compiled tile shapes (S strips x BN channels):
//   (25, 64):  the whole sample at 384 < T <= 400 (C3's 256-wide stage: 256 tiles);
//   (32, 64):  500-row tiles at T = 2000 (tm in (496, 512]; 512 tiles at C3);
//   (16, 128): 250-row tiles x 128 channels at T = 2000 (tm in (240, 256]): the
//              input ELU once per 128 output channels instead of twice, for the
//              ELU'd forwards (the RU128 k7 convs; 512 tiles at C3).
// tune key 51: 1 = (16, 128) wherever it applies, 2 = never, 0 = for in_elu only
// samples per tile: 400 / T for the short sequences whole 16-row strips tile
// exactly (T = 80 at C3: five samples per 25-strip tile); tune key 67 = 2: never
// (the dispatch takes them only under key 67 = 1 / 3, conv.hip wss_pick_short)
int wss_spt(const Args& a) {
  return (a.T % 16 == 0 && a.T >= 80 && a.T < 400 && 400 % a.T == 0 && tune(67) != 2) ? 400 / a.T : 1;
}

bool wss_geometry(const Args& a, int& S, int& tm, int& BN) {
  BN = 64;
  const int S1 = (a.T + 15) / 16;
  if (S1 == 25 || wss_spt(a) > 1) {
    S = 25;
    tm = S1 == 25 ? a.T : 400;
    return true;
  }
  const int k51 = tune(51);
  if (a.N % 128 == 0 && (k51 == 1 || (k51 == 0 && a.in_elu))) {
    const int n = (a.T + 255) / 256;
    const int t = (a.T + n - 1) / n;
    if ((t + 15) / 16 == 16) {
      S = 16;
      tm = t;
      BN = 128;
      return true;
    }
  }
  const int ntps = (a.T + 511) / 512;
  tm = (a.T + ntps - 1) / ntps;
  S = (tm + 15) / 16;
  return S == 32;
}

bool wss_geometry(const Args& a, int& S, int& tm) {
  int BN;
  return wss_geometry(a, S, tm, BN);
}

bool wss_ok(const Args& a) {
  int S, tm, BN;
  const bool kt = a.K == 7 || a.K == 3 || a.K == 2;
  return kt && wss_geometry(a, S, tm, BN) && a.N % BN == 0 && a.C % (2 * WSS_CK) == 0 && a.C <= WSS_CMAX &&
         (a.K - 1) * a.dil <= F4_HALOMAX && a.pad <= (a.K - 1) * a.dil && a.seq_pitch == 0 && a.epi == 0 &&
         a.tin_valid == a.T && a.tin_pitch == a.T && a.tout_valid == a.T && a.ldx == a.C && a.ldo == a.N &&
         a.rows % a.T == 0;
}

template <int KT, int S, int BN, typename TO, int SPT = 1>
static int launch_wss_t(const Args& a, int tm, const void* in, const void* wp, const float* bias, const void* aux,
                        const void* res, void* out, hipStream_t s) {
  using G = WssGeo<KT, S, BN, SPT>;
  static_assert(G::LDS <= 160 * 1024, "LDS");
  const int64_t tiles = SPT == 1 ? (a.rows / a.T) * ((a.T + tm - 1) / tm) : (a.rows / a.T + SPT - 1) / SPT;
  const int ncol = a.N / BN;
  if (tiles == 0) return SEL_OK;
  SEL_REQUIRE(tiles * ncol < (int64_t(1) << 31), SEL_ERR_UNSUPPORTED, "k_conv_wss: grid too large");
  auto kern = k_conv_wss<KT, S, BN, TO, SPT>;
  SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(G::LDS)));
  hipLaunchKernelGGL(kern, dim3(unsigned(tiles * ncol)), dim3(512), G::LDS, s, a, static_cast<const __bf16*>(in),
                     static_cast<const __bf16*>(wp), bias, static_cast<const TO*>(aux), static_cast<const TO*>(res),
                     static_cast<TO*>(out), ncol, tm, tune(48), nullptr, nullptr, nullptr);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <int S, int BN, typename TO, int SPT = 1>
static int launch_wss_k(const Args& a, int tm, const void* in, const void* wp, const float* bias, const void* aux,
                        const void* res, void* out, hipStream_t s) {
  switch (a.K) {
    case 7: return launch_wss_t<7, S, BN, TO, SPT>(a, tm, in, wp, bias, aux, res, out, s);
    case 3: return launch_wss_t<3, S, BN, TO, SPT>(a, tm, in, wp, bias, aux, res, out, s);
    default: return launch_wss_t<2, S, BN, TO, SPT>(a, tm, in, wp, bias, aux, res, out, s);
  }
}

template <typename TO>
int launch_wss(const Args& a, const void* in, const void* wp, const float* bias, const void* aux, const void* res,
               void* out, hipStream_t s) {
  SEL_REQUIRE(wss_ok(a), SEL_ERR_ARG, "k_conv_wss: unsupported shape T=%d C=%d N=%d K=%d dil=%d", a.T, a.C, a.N,
              a.K, a.dil);
  int S, tm, BN;
  wss_geometry(a, S, tm, BN);
  if (S == 25 && wss_spt(a) == 5) return launch_wss_k<25, 64, TO, 5>(a, tm, in, wp, bias, aux, res, out, s);
  if (S == 25 && wss_spt(a) == 1) return launch_wss_k<25, 64, TO>(a, tm, in, wp, bias, aux, res, out, s);
  SEL_REQUIRE(S != 25, SEL_ERR_UNSUPPORTED, "k_conv_wss: %d samples per tile not compiled", wss_spt(a));
  if constexpr (sizeof(TO) == 2) {  // (fp32 outputs: the epilogue rows do not fit the taller tiles' registers)
    if (S == 16) return launch_wss_k<16, 128, TO>(a, tm, in, wp, bias, aux, res, out, s);
    return launch_wss_k<32, 64, TO>(a, tm, in, wp, bias, aux, res, out, s);
  }
  set_error("k_conv_wss: fp32 output needs T <= 400");
  return SEL_ERR_UNSUPPORTED;
}

// the fused 128-channel residual-unit forward (RU epilogue): conv1 = `a` (C = N
// = 128, K = 7, causal zero pad, ELU prologue) on the (16, 128) tile
bool wss_pw_ok(const Args& a) {
  int S, tm, BN;
  return a.C == 128 && a.N == 128 && a.K == 7 && a.in_elu == 1 && a.pad == 6 * a.dil &&
         a.pad_mode == SEL_PAD_ZERO && (a.bias_period == 0 || a.bias_period == a.N) && tune(69) != 1 &&
         wss_ok(a) && wss_geometry(a, S, tm, BN) && S == 16 && BN == 128;
}

int launch_wss_pw(const Args& a, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                  void* h, void* out, hipStream_t s) {
  SEL_REQUIRE(wss_pw_ok(a), SEL_ERR_UNSUPPORTED, "k_conv_wss RU: unsupported shape T=%d C=%d dil=%d", a.T, a.C,
              a.dil);
  int S, tm, BN;
  wss_geometry(a, S, tm, BN);
  using G = WssGeo<7, 16, 128>;
  const int64_t tiles = (a.rows / a.T) * ((a.T + tm - 1) / tm);
  if (tiles == 0) return SEL_OK;
  SEL_REQUIRE(tiles < (int64_t(1) << 31), SEL_ERR_UNSUPPORTED, "k_conv_wss: grid too large");
  auto kern = k_conv_wss<7, 16, 128, __bf16, 1, true>;
  SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(G::LDS)));
  hipLaunchKernelGGL(kern, dim3(unsigned(tiles)), dim3(512), G::LDS, s, a, static_cast<const __bf16*>(x),
                     static_cast<const __bf16*>(w1), b1, static_cast<const __bf16*>(nullptr),
                     static_cast<const __bf16*>(x), static_cast<__bf16*>(h), 1, tm, tune(48) & ~16,
                     static_cast<const __bf16*>(w2), b2, static_cast<__bf16*>(out));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

bool wss_ok_out(const Args& a, bool out_f32) {
  int S, tm;
  return wss_ok(a) && (!out_f32 || (wss_geometry(a, S, tm) && S == 25));
}

template int launch_wss<__bf16>(const Args&, const void*, const void*, const float*, const void*, const void*, void*,
                                hipStream_t);
template int launch_wss<float>(const Args&, const void*, const void*, const float*, const void*, const void*, void*,
                               hipStream_t);

}  // namespace conv
}  // namespace sel
