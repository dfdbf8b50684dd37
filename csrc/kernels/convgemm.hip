// Convolutions of NHWC (channels_last) bf16 activations as implicit MFMA GEMMs, with the
// neighbouring BatchNorm passes folded into their prologues / epilogues -- the ResNet-50
// bottleneck (im2col + conv GEMM + weight gradient, MI355X-native).
//
// Output pixel m = (i, oh, ow) reads input pixel (i, oh*s - p + kh, ow*s - p + kw) for tap
// (kh, kw); the reduction index is k = (kh*ks + kw)*C + c, so the channels_last weight
// [N][ks][ks][C] is already the K-contiguous B operand and no im2col buffer exists: the
// staging loads gather A rows tap by tap (C % 64 == 0: a 64-deep stage never straddles taps).
//
// At ResNet-50 widths most 1x1 layers are HBM-bound (2MKN FLOPs against 2M(K+N) bytes), so the
// lever is the number of passes over the activations.  Each GEMM folds adjacent BN work in:
//
//   conv_fwd    C[m, n] = sum_k f(A[src(m, k)]) B[n, k]   (forward; the data gradient is the
//               same GEMM on the transposed / flipped weight)
//     prologue  f(a) = relu(a * scale_c + shift_c): the previous BN + ReLU applied while A is
//               staged -- that BN's output is never written (taps outside the map stay 0)
//     epilogue  1: per-channel partial sums of C about a shift (the next BN's statistics)
//               2: + residual rows (block-input gradient = conv1 data grad + identity grad)
//               3: ReLU mask from z*scale + shift and that BN's backward sums sum(g),
//                  sum(g * xhat) -- its reduce pass
//               4: + a stride-2 map's rows at even (h, w) (downsample data gradient)
//               5: + residual rows masked by forward ReLU bits (identity gradient, never stored)
//               6/7/8: epilogue 5/2/4, then the PREVIOUS block's bn3 backward reduce folded in:
//                  g = v * relu'(previous block output) from its bits (stored masked) and the
//                  sums sum(g), sum(g * (z3 - mean) * invstd) over that block's bn3 input z3
//               9: epilogue 6 when the previous block has a downsample branch: its BN's backward
//                  gets the same g, so a third sum sum(g * (zd - mean2) * invstd2) over the
//                  downsample BN input zd replaces that BN's separate reduce pass
//   conv_wgrad  dW[n, k] = sum_m dZ[m, n] f(A[src(m, k)]), split over m; both operands are read
//               transposed from row-major LDS tiles (ds_read_b64_tr_b16); fp32 per-split slabs,
//               fixed-order reduction (deterministic, no atomics).
//
// MFMA v_mfma_f32_32x32x16_bf16 with the weight tile as the A operand, so every lane's
// accumulator holds 4 consecutive output channels of one pixel; the tile goes through LDS and
// leaves as 16-byte row pieces, which is also where the epilogue statistics are taken (on the
// bf16-rounded values the next BN reads).  The forward grid is persistent (2 blocks per CU, a
// fixed channel tile per block), so the statistics accumulate in registers across pixel tiles
// and the BN finalize kernels sum only [2][blocks][N] partials in fixed order.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kBM = 128;  // output pixels per tile (conv_fwd)
constexpr int kBK = 64;   // reduction depth per LDS stage: 8 x 16-B chunks per row
constexpr int kWM = 64;   // pixels per LDS stage (conv_wgrad)

__device__ __forceinline__ bf16x8_t as_bf16x8(s16x8 v) { return __builtin_bit_cast(bf16x8_t, v); }

// LDS hand-off barrier that waits for this wave's LDS traffic only; __syncthreads() would also
// drain the prefetched stage's global loads.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Bijective XCD-aware remap (blocks b and b + 8 share an XCD): consecutive logical ids run on
// one XCD, so the channel tiles of one pixel tile share its A rows through that XCD's L2.
__device__ __forceinline__ int xcd_remap(int b, int nblk) {
  const int q = nblk >> 3, r = nblk & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// Source of output pixel m: image (-1 past M) and the input coordinates of tap (0, 0).
struct PixSrc {
  int img, ih0, iw0;
};

__device__ __forceinline__ PixSrc pix_src(int m, int M, const ConvGeo& g) {
  PixSrc s{-1, 0, 0};
  if (m < M) {
    const int ohw = g.OH * g.OW;
    s.img = m / ohw;
    const int r = m - s.img * ohw, oh = r / g.OW;
    s.ih0 = oh * g.stride - g.pad;
    s.iw0 = (r - oh * g.OW) * g.stride - g.pad;
  }
  return s;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) { return (__umulhi(n, f.mul) + n) >> f.shift; }

// pix_src with the two divisions by invariant divisors done as multiply-high + shift
__device__ __forceinline__ PixSrc pix_src_fd(int m, int M, const ConvGeo& g, const FastDiv& fohw,
                                            const FastDiv& fow) {
  PixSrc s{-1, 0, 0};
  if (m < M) {
    s.img = static_cast<int>(fdiv(static_cast<uint32_t>(m), fohw));
    const int r = m - s.img * (g.OH * g.OW);
    const int oh = static_cast<int>(fdiv(static_cast<uint32_t>(r), fow));
    s.ih0 = oh * g.stride - g.pad;
    s.iw0 = (r - oh * g.OW) * g.stride - g.pad;
  }
  return s;
}

// Element offset of channel c of tap (kh, kw) of pixel s, or -1 outside the map / past M.
__device__ __forceinline__ int64_t tap_off(const PixSrc& s, int kh, int kw, int c, const ConvGeo& g) {
  const int ih = s.ih0 + kh, iw = s.iw0 + kw;
  if (s.img < 0 || static_cast<unsigned>(ih) >= static_cast<unsigned>(g.H) ||
      static_cast<unsigned>(iw) >= static_cast<unsigned>(g.W))
    return -1;
  return ((static_cast<int64_t>(s.img) * g.H + ih) * g.W + iw) * g.C + c;
}

// [rows][64] tiles read as ds_read_b128 fragments: 16-B chunk c of row r is stored at chunk
// c ^ ((r >> 1) & 7), so every 16-lane group of a fragment read (rows {0-3,12-15,20-27} or
// {4-11,16-19,28-31} of a 32-row block, one chunk) hits 16 distinct bank slots.
__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 7); }

// [64][RL] tiles read transposed (ds_read_b64_tr_b16): a 32-lane half reads rows r0..r0+3 x 64
// contiguous bytes; the chunk XOR gives each of the 4 rows its own quarter of the bank row.
template <int RL>
__device__ __forceinline__ int tr_swz(int r) {
  return RL >= 128 ? (r & 3) << 2 : ((r >> 1) & 1) << 2;  // rows of >= 256 B / 128 B
}
template <int RL>
__device__ __forceinline__ int tr_off(int r, int col) {
  return r * RL + ((col >> 3) ^ tr_swz<RL>(r)) * 8 + (col & 7);
}

// 32x32x16 MFMA operand from a [64][RL] tile read transposed: lane l receives
// T[16 s + 8 (l >> 5) + j][c0 + (l & 31)], j = 0..7 (two 4-row transposed reads; lane 4q + p of
// each 16-lane group addresses row q, columns 4p..4p+3 of its block).
template <int RL>
__device__ __forceinline__ bf16x8_t tr_frag(const uint16_t* T, int s, int c0, int lane) {
  const int gi = lane >> 4, i16 = lane & 15;
  const int r = 16 * s + 8 * (gi >> 1) + (i16 >> 2);
  const int col = c0 + 16 * (gi & 1) + 4 * (i16 & 3);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(T + tr_off<RL>(r, col)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(T + tr_off<RL>(r + 4, col)));
  return as_bf16x8(s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
}

// tr_frag through inline asm: the compiler cannot tell an LDS-DMA (global_load_lds) in flight to
// the other buffer from this read and would put s_waitcnt vmcnt(0) before every ds_read_b64_tr_b16
// (serialising the prefetch).  The caller waits lgkmcnt itself (lds_wait_frags).
template <int RL>
__device__ __forceinline__ bf16x8_t tr_frag_asm(const uint16_t* T, int s, int c0, int lane) {
  const int gi = lane >> 4, i16 = lane & 15;
  const int r = 16 * s + 8 * (gi >> 1) + (i16 >> 2);
  const int col = c0 + 16 * (gi & 1) + 4 * (i16 & 3);
  const unsigned a0 = static_cast<unsigned>(reinterpret_cast<uintptr_t>((const lds_s16x4*)(T + tr_off<RL>(r, col))));
  const unsigned a1 = static_cast<unsigned>(reinterpret_cast<uintptr_t>((const lds_s16x4*)(T + tr_off<RL>(r + 4, col))));
  s16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a0) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(a1) : "memory");
  return as_bf16x8(s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
}

// tr_frag with the lane's address precomputed (tr_frag_base) and the k-step / half-row offsets as
// instruction immediates: no per-fragment address arithmetic inside the MFMA loop.
template <int RL>
__device__ __forceinline__ uint32_t tr_frag_base(int c0, int lane) {
  const int gi = lane >> 4, i16 = lane & 15;
  const int r = 8 * (gi >> 1) + (i16 >> 2);
  const int col = c0 + 16 * (gi & 1) + 4 * (i16 & 3);
  return static_cast<uint32_t>(tr_off<RL>(r, col) * 2);
}
template <int RL, int S>
__device__ __forceinline__ bf16x8_t tr_frag_imm(uint32_t addr) {
  // rows 16 S + r and 16 S + r + 4 share the lane's swizzle (tr_swz looks at r & 3 / (r >> 1) & 1)
  constexpr int o0 = S * 16 * RL * 2, o1 = o0 + 4 * RL * 2;
  s16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(addr), "i"(o0) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(addr), "i"(o1) : "memory");
  return as_bf16x8(s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
}

// relu(bf16(x * scale + shift)): the ReLU runs on the packed bf16 result as signed 16-bit
// integers (every negative bf16, -0 included, has the sign bit set, so max(., 0) as int16 is the
// bf16 ReLU) -- one v_pk_max_i16 per pair instead of a float max per element; identical results
// (rounding a negative value never makes it positive)
typedef short s16x8i __attribute__((ext_vector_type(8)));
__device__ __forceinline__ u16x8 bn_relu8(u16x8 v, const float (&sc)[8], const float (&sh)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f32_to_bf16(bf16_to_f32(v[j]) * sc[j] + sh[j]);
  const s16x8i z = {0, 0, 0, 0, 0, 0, 0, 0};
  return __builtin_bit_cast(u16x8, __builtin_elementwise_max(__builtin_bit_cast(s16x8i, v), z));
}

constexpr u16x8 kZero8 = {0, 0, 0, 0, 0, 0, 0, 0};

typedef __attribute__((address_space(1))) const void gptr_t;
typedef __attribute__((address_space(3))) void lptr_t;

}  // namespace

// source of the LDS-DMA loads of out-of-map taps / rows past M
__device__ __attribute__((aligned(16))) uint16_t kZeroPage[8] = {0, 0, 0, 0, 0, 0, 0, 0};

// ------------------------------------------------------------------------------ conv_fwd
// Persistent grid of nN * GM blocks of 256 threads (4 waves: 2 pixel halves x 2 channel halves):
// block (n-tile nt, group mg) computes pixel tiles mg, mg + GM, ... of channel tile nt (a fixed
// channel tile, so the epilogue statistics stay in registers across tiles and the partials are
// [2][GM][N]).  Tile 128 pixels x BN channels; K in 64-deep stages.  The block walks one linear
// sequence of (tile, stage) steps through two LDS buffers and two register stage sets: the loads
// of step q + 2 are issued before the MFMAs of step q, so two steps of work -- and at tile ends
// the epilogue -- cover their latency (the HBM-bound 1x1 layers have a single stage per tile).
template <int AR, int BCH, int AR2>
struct StageRegs {
  u16x8 a[AR];
  u16x8 a2[AR2];  // BN-backward prologue: the BN input rows (AR2 = 1: unused)
  u16x8 b[BCH];
  int mt;         // pixel tile of the stage (BN-backward prologue: where the A tile is stored)
  unsigned ok;  // valid-row bits of a[]
  int cc;       // channel offset of the stage inside its tap (prologue coefficients)
  bool wb;      // b[] loaded (to be staged)
};

// PRO: 0 none, 1 BN + ReLU of the A rows, 2 BN backward from two row sources (a, a2),
// 3 the previous block's output relu(bn3(a) + r) with r = a2 (identity) or bnd(a2) (downsample)
// PATCH (3x3 / stride 1 / pad 1, LDS-DMA path): the tile's input rows -- a PATCH of whole rows with
// zero halo rows / columns, at most two images -- are staged ONCE per 64-channel chunk and the nine
// taps read their A fragments from it at a shifted slot; a K stage then moves only its weight tile.
// The im2col staging moved 9 copies of every input pixel through L2 (52 FLOP per staged byte on
// the 64-channel layers: L2-bandwidth bound).  Patch layout: eight 16-B channel planes of
// [rows][W + 2] slots, so 16 consecutive pixels of a b128 fragment read hit 16 distinct rows.
template <int BN>
constexpr int patch_bytes() { return BN == 64 ? 65536 : 40960; }  // 8 channel planes of 8 / 5 KiB

// VAR: 0 the plain paths, 1 PATCH (3x3 patch-staged tiles).  (A 3-stage ring for the plain
// LDS-DMA path measured no faster: profiles/r4_deep_ring_graph_ab.txt; removed in round 6.)
// The kernel body takes its logical block id L (XCD-remapped) from the launching kernel: conv_fwd_kernel
// (one GEMM per launch) or conv_dgrad_phases_kernel (the four stride-2 data-gradient phases in one grid).
template <int BM, int BN, int PRO, int EPI, bool KS1, bool GLDS, int VAR = 0>
__device__ __forceinline__ void conv_fwd_body(const ConvGemmArgs& p, int GM, int L) {
  constexpr bool BWD = PRO == 2;
  constexpr bool RESP = PRO == 3;
  static_assert(!BWD || (KS1 && EPI == 3), "the BN-backward prologue is a 1x1 data-gradient prologue");
  static_assert(!RESP || (KS1 && EPI <= 1), "the block-output prologue is a 1x1 forward prologue");
  // two-source prologues on the LDS-DMA path: both row sources land in LDS by DMA and one pass
  // over the stage tile applies the prologue in place (a single third buffer for the second
  // source: it is refilled once the pass has read it)
  constexpr bool TWO_GLDS = GLDS && (BWD || RESP);
  // PRO 1 (BN + ReLU of A) on the LDS-DMA path: the same in-place pass, one source (1x1 only:
  // the pass cannot tell a 3x3 halo slot's zero from a real 0)
  constexpr bool ONE_GLDS = GLDS && PRO == 1;
  static_assert(!ONE_GLDS || KS1, "the LDS-pass BN prologue is for 1x1 convolutions");
  constexpr bool XF_GLDS = TWO_GLDS || ONE_GLDS;
  constexpr int AR2 = BWD || RESP ? BM / 32 : 1;
  // epilogues 6/7/8 = base epilogue 5/2/4 + the previous block's bn3 backward reduce; 9 = 6 + the
  // previous block's downsample-BN sum (third partial slab)
  constexpr bool FOLD = EPI >= 6;
  constexpr bool FOLD_DS = EPI == 9;
  constexpr int BASE = EPI == 6 || EPI == 9 ? 5 : EPI == 7 ? 2 : EPI == 8 ? 4 : EPI;
  constexpr int NSUM = FOLD_DS ? 3 : 2;
  // waves 2 x 2 over the tile; the tall 256 x 64 tile (LDS-DMA path only) stacks them 4 x 1 so
  // every wave still computes 64 x 64 (a 128 x 64 tile gave each wave 64 x 32: 1.5 fragment
  // reads per MFMA instead of 1, and half the weight-tile reuse)
  constexpr bool TALL = BM == 256;
  static_assert(!TALL || (BN == 64 && GLDS), "the 256-pixel tile is the LDS-DMA 64-channel variant");
  constexpr int TN = TALL ? BN / 32 : BN / 64;  // 32-channel MFMA blocks per wave
  constexpr int TM = TALL ? 2 : BM / 64;        // 32-pixel MFMA blocks per wave
  constexpr int AR = BM / 32;              // A-tile chunks per thread per stage
  constexpr int BCH = BN / 32;             // B-tile chunks per thread per stage
  constexpr int BI_P = BN / 32;            // PATCH: weight LDS-DMA instructions per wave per stage
  // output tile row stride (bf16): 2 dwords mod 32 banks, so the 16 rows of a ds_write_b64 lane
  // group hit distinct bank pairs (BN + 8 made them 2-way); rows are 8-B aligned -> b64 readback
  constexpr int CS = BN + 4;
  // LDS: [A0 | A1] overlaid by the output tile + statistics scratch, then [B0 | B1] (never
  // overlaid, so a resident weight tile survives the epilogues)
  // EPI 9 keeps its third running sum in LDS (8 floats per thread past the output tile): in
  // registers it pushed the register-staged variant from 20 to 76 B/lane of scratch
  constexpr int RED_ELEMS = 4 * NSUM * BN * 2 > (FOLD_DS ? 256 * 8 * 2 : 0) ? 4 * NSUM * BN * 2 : 256 * 8 * 2;
  constexpr int EPI_ELEMS = BM * CS + RED_ELEMS;
  constexpr bool PATCH = VAR == 1;
  constexpr int NST = 2;  // LDS-DMA ring depth
  static_assert(VAR == 0 || VAR == 1, "plain or patch");
  constexpr int A_ELEMS = PATCH ? patch_bytes<BN>() / 2 : (TWO_GLDS ? 3 : NST) * BM * kBK;
  constexpr int Z_BASE = 2 * BM * kBK;  // TWO_GLDS: the second source's stage tile
  constexpr int B_BASE = ((A_ELEMS > EPI_ELEMS ? A_ELEMS : EPI_ELEMS) + 7) & ~7;
  constexpr int LDS_ELEMS = B_BASE + NST * BN * kBK;
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_ELEMS];

  const ConvGeo& g = p.g;
  // wave id through readfirstlane: provably uniform, so LDS-DMA destinations (M0) and other
  // per-wave addresses stay in SGPRs instead of VALU + v_readfirstlane per instruction
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nN = p.N / BN, mtiles = (p.M + BM - 1) / BM;
  const int mg = L / nN, n0 = (L - mg * nN) * BN;
  if (mg >= GM) return;  // (block-uniform) padding blocks of a phase-merged grid
  const int nk = p.K / kBK;
  const int my_tiles = mg < mtiles ? (mtiles - mg + GM - 1) / GM : 0;
  const int nq = my_tiles * nk;  // block-uniform

  // staging: thread t moves 16-B chunk (t & 7) of tile rows (t >> 3) + 32 i
  const int srow = t >> 3, sc = t & 7;
  const uint16_t* bptr = p.b + static_cast<int64_t>(n0 + srow) * p.K + sc * 8;
  StageRegs<AR, BCH, AR2> S0, S1;
  // producer cursor (runs two steps ahead of the MFMAs): tile iteration pti, stage pkt and its
  // tap (pkh, pkw) / channel offset pcc, advanced incrementally (no divisions per stage);
  // per-tile row sources: offset of tap (0, 0) channel 0, its input coordinates, row valid
  int pti = 0, pkt = 0, pkh = 0, pkw = 0, pcc = 0;
  // with <= 2 stages per tile, buffer (q & 1) always holds the same k-stage, so its weight tile
  // is staged by the first two steps only and stays resident
  int lq = 0;
  int64_t rbase[AR];
  int rih[AR], riw[AR];
  unsigned rok = 0;
  auto set_rows = [&](int mt) {
    rok = 0;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const PixSrc ps = pix_src_fd(mt * BM + srow + 32 * i, p.M, g, p.fd_ohw, p.fd_ow);
      rok |= (ps.img >= 0 ? 1u : 0u) << i;
      rih[i] = ps.ih0;
      riw[i] = ps.iw0;
      rbase[i] = ((static_cast<int64_t>(ps.img > 0 ? ps.img : 0) * g.H + ps.ih0) * g.W + ps.iw0) * g.C + sc * 8;
    }
  };
  auto gload = [&](StageRegs<AR, BCH, AR2>& R) {
    R.cc = pcc;
    R.ok = 0;
    R.mt = mg + pti * GM;
    const int64_t toff = KS1 ? pcc : static_cast<int64_t>(pkh * g.W + pkw) * g.C + pcc;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      bool v = (rok >> i) & 1u;
      if constexpr (!KS1) {
        v = v && static_cast<unsigned>(rih[i] + pkh) < static_cast<unsigned>(g.H) &&
            static_cast<unsigned>(riw[i] + pkw) < static_cast<unsigned>(g.W);
      }
      R.ok |= (v ? 1u : 0u) << i;
      // out-of-map taps / rows past M read element 0 (in bounds) and are zeroed in LDS
      R.a[i] = *reinterpret_cast<const u16x8*>(p.a + (v ? rbase[i] + toff : 0));
      if constexpr (BWD || RESP) R.a2[i] = *reinterpret_cast<const u16x8*>(p.a2 + (v ? rbase[i] + toff : 0));
    }
    const int k0 = pkt * kBK;
    R.wb = lq++ < 2 || nk > 2;
    if (R.wb) {
#pragma unroll
      for (int i = 0; i < BCH; ++i)
        R.b[i] = *reinterpret_cast<const u16x8*>(bptr + static_cast<int64_t>(32 * i) * p.K + k0);
    }
    // advance the cursor
    pcc += kBK;
    if (pcc == g.C) {
      pcc = 0;
      if (++pkw == (g.ksw ? g.ksw : g.ks)) {
        pkw = 0;
        ++pkh;
      }
    }
    if (++pkt == nk) {
      pkt = pkh = pkw = pcc = 0;
      if (++pti < my_tiles) set_rows(mg + pti * GM);
    }
  };
  auto swrite = [&](const StageRegs<AR, BCH, AR2>& R, int buf) {
    uint16_t* As = lds + buf * (BM * kBK);
    uint16_t* Bs = lds + B_BASE + buf * (BN * kBK);
    float psc[8], psh[8], pcf[8], pdd[8];
    if constexpr (PRO == 1 || RESP) {  // [scale | shift] of 8 channels: L1-resident
      load8(p.pro, R.cc + sc * 8, psc);
      load8(p.pro + g.C, R.cc + sc * 8, psh);
    } else if constexpr (BWD) {  // [ca | cb | cc]
      load8(p.bwd, R.cc + sc * 8, psc);
      load8(p.bwd + g.C, R.cc + sc * 8, psh);
      load8(p.bwd + 2 * g.C, R.cc + sc * 8, pcf);
    }
    const bool dual = RESP && p.pro2 != nullptr;  // block-uniform
    if (dual) {  // the downsample BN's [scale | shift]
      load8(p.pro2, R.cc + sc * 8, pcf);
      load8(p.pro2 + g.C, R.cc + sc * 8, pdd);
    }
    // BWD / RESP: the channel-tile-0 blocks also store the A tile (the BN data gradient / the
    // block output, with its ReLU bits) to aout
    const bool store_a = (BWD || RESP) && p.aout != nullptr && n0 == 0;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      u16x8 v = R.a[i];
      if constexpr (PRO == 1) v = bn_relu8(v, psc, psh);
      if constexpr (BWD) {
        const u16x8 x8 = R.a2[i];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = f32_to_bf16(psc[j] * bf16_to_f32(v[j]) + psh[j] * bf16_to_f32(x8[j]) + pcf[j]);
      }
      unsigned obits = 0;
      if constexpr (RESP) {  // the same arithmetic as bn_apply_kernel / bn_apply_dual_kernel
        const u16x8 r8 = R.a2[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float o = bf16_to_f32(v[j]) * psc[j] + psh[j];
          if (dual) o = o + (bf16_to_f32(r8[j]) * pcf[j] + pdd[j]);
          else o += bf16_to_f32(r8[j]);
          o = o > 0.f ? o : 0.f;
          obits |= (o > 0.f ? 1u : 0u) << j;
          v[j] = f32_to_bf16(o);
        }
      }
      const bool ok = (R.ok >> i) & 1u;
      if (!ok) v = kZero8;
      const int r = srow + 32 * i;
      *reinterpret_cast<u16x8*>(As + r * kBK + swz(r, sc) * 8) = v;
      if (store_a && ok) {
        const int64_t e = static_cast<int64_t>(R.mt * BM + r) * g.C + R.cc + sc * 8;
        *reinterpret_cast<u16x8*>(p.aout + e) = v;
        if constexpr (RESP) p.abits[e >> 3] = static_cast<uint8_t>(obits);
      }
    }
    if (R.wb) {
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        const int r = srow + 32 * i;
        *reinterpret_cast<u16x8*>(Bs + r * kBK + swz(r, sc) * 8) = R.b[i];
      }
    }
  };

  const int wm = TALL ? wave * 64 : (wave >> 1) * (BM / 2), wn = TALL ? 0 : (wave & 1) * (BN / 2);
  const int fr = lane & 31, fh = lane >> 5;
  f32x16 acc[TN][TM];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  };
  auto compute = [&](int buf) {
    const uint16_t* As = lds + buf * (BM * kBK);
    const uint16_t* Bs = lds + B_BASE + buf * (BN * kBK);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ch = 2 * s + fh;  // this lane's chunk: k = 16 s + 8 fh + j
      bf16x8_t xa[TM], wb[TN];
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int r = wm + 32 * j + fr;
        xa[j] = *reinterpret_cast<const bf16x8_t*>(As + r * kBK + swz(r, ch) * 8);
      }
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int r = wn + 32 * i + fr;
        wb[i] = *reinterpret_cast<const bf16x8_t*>(Bs + r * kBK + swz(r, ch) * 8);
      }
      // D[n][m] = sum_k W[n][k] A[m][k]: the weight rows are the MFMA A operand
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wb[i], xa[j], acc[i][j], 0, 0, 0);
    }
  };

  // output pass: thread t owns channels [8 cg, 8 cg + 8) of tile rows r0, r0 + RPP, ...
  constexpr int CPR = BN / 8, RPP = 256 / CPR;
  const int cg = t % CPR, r0 = t / CPR, nc = n0 + cg * 8;
  float s1[8], s2[8], e0[8], e1[8], e2[8], e3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = e0[j] = e1[j] = e2[j] = e3[j] = 0.f;
  float* s3l = reinterpret_cast<float*>(lds + BM * CS) + t * 8;  // EPI 9: this thread's third sum
  if constexpr (FOLD_DS) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s3l[j] = 0.f;
  }
  if constexpr (EPI == 1) {
    if (p.kshift) load8(p.kshift, nc, e0);
  } else if constexpr (EPI == 3) {
    load8(p.mc, nc, e0);
    load8(p.mc + p.N, nc, e1);
    load8(p.mean, nc, e2);
    load8(p.invstd, nc, e3);
  } else if constexpr (FOLD) {
    load8(p.mean, nc, e2);
    load8(p.invstd, nc, e3);
  }
  uint16_t* Cs = lds;
  // Epilogue reads (residual / BN-input / mask rows of this thread's NPASS output rows), issued
  // together before any is consumed: a load-use loop paid one HBM latency per row (the read-heavy
  // data-gradient epilogues ran at ~2.8 TB/s).  Rows past M read row M - 1 (in bounds, unused).
  constexpr int NPASS = BM / RPP;
  // destination row of output pixel m (a stride-2 data-gradient phase scatters to every other row)
  // (only the phase launches -- epilogues 0 / 3, bindings conv_dgrad_s2 -- carry RH > 0: the
  // other epilogues compile the scatter away)
  auto orow = [&](int m) -> int64_t {
    if (!(EPI == 0 || EPI == 3) || g.RH == 0) return m;
    const int ohw = g.OH * g.OW, im = static_cast<int>(fdiv(static_cast<uint32_t>(m), p.fd_ohw)), r = m - im * ohw,
              i = static_cast<int>(fdiv(static_cast<uint32_t>(r), p.fd_ow)), j = r - i * g.OW;
    return (static_cast<int64_t>(im) * g.RH + 2 * i + g.ra) * g.RW + 2 * j + g.rb;
  };
  constexpr bool RD_AUX = BASE == 5 || BASE == 2 || BASE == 4 || EPI == 3;
  u16x8 ra[RD_AUX ? NPASS : 1], rz[FOLD ? NPASS : 1];
  unsigned rb[BASE == 5 ? NPASS : 1], rp[FOLD ? NPASS : 1];
  unsigned rodd = 0;  // BASE 4: rows without a residual (odd h or w)
  auto epi_load = [&](int mt) {
    const int m0 = mt * BM;
    rodd = 0;
#pragma unroll
    for (int i = 0; i < NPASS; ++i) {
      const int m = min(m0 + r0 + i * RPP, p.M - 1);
      const int64_t o = orow(m) * p.N + nc;
      if constexpr (BASE == 4) {  // residual map (OH+1)/2 x (OW+1)/2, present at even (h, w)
        const int ohw = g.OH * g.OW;
        const int im = static_cast<int>(fdiv(static_cast<uint32_t>(m), p.fd_ohw)), r = m - im * ohw,
                  h = static_cast<int>(fdiv(static_cast<uint32_t>(r), p.fd_ow)), w = r - h * g.OW;
        const int RH = (g.OH + 1) >> 1, RW = (g.OW + 1) >> 1;
        ra[i] = kZero8;
        rodd |= static_cast<unsigned>((h | w) & 1) << i;
        if (!((h | w) & 1))
          ra[i] = *reinterpret_cast<const u16x8*>(
              p.aux + ((static_cast<int64_t>(im) * RH + (h >> 1)) * RW + (w >> 1)) * p.N + nc);
      } else if constexpr (RD_AUX) {
        ra[i] = *reinterpret_cast<const u16x8*>(p.aux + o);
      }
      if constexpr (BASE == 5) rb[i] = p.bits[o >> 3];
      if constexpr (FOLD) {
        rz[i] = *reinterpret_cast<const u16x8*>(p.aux2 + o);
        rp[i] = p.bits2[o >> 3];
      }
    }
  };
  // accumulators -> bf16 output tile [BM][CS]: register q of lane l is channel
  // (q & 3) + 8 (q >> 2) + 4 (l >> 5), pixel l & 31 -> 4 consecutive channels per 8-B store
  auto acc_to_lds = [&]() {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j)
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const int nl = wn + 32 * i + 8 * q4 + 4 * fh, ml = wm + 32 * j + fr;
          const u16x4 v = {f32_to_bf16(acc[i][j][4 * q4]), f32_to_bf16(acc[i][j][4 * q4 + 1]),
                           f32_to_bf16(acc[i][j][4 * q4 + 2]), f32_to_bf16(acc[i][j][4 * q4 + 3])};
          *reinterpret_cast<u16x4*>(Cs + ml * CS + nl) = v;
        }
  };
  // epilogue_rows(mt) consumes what epi_load(mt) read, from the output tile acc_to_lds() wrote
  auto epilogue_rows = [&](int mt) {
    const int m0 = mt * BM;
#pragma unroll
    for (int i = 0; i < NPASS; ++i) {
      const int rr = r0 + i * RPP, m = m0 + rr;
      if (m >= p.M) break;
      const u16x4 lo = *reinterpret_cast<const u16x4*>(Cs + rr * CS + cg * 8);
      const u16x4 hi = *reinterpret_cast<const u16x4*>(Cs + rr * CS + cg * 8 + 4);
      u16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const int64_t o = orow(m) * p.N + nc;
      if constexpr (BASE == 5) {  // identity-branch gradient = dout * relu'(block output), from bits
        v = bf16_add_where(v, ra[i], rb[i]);
      } else if constexpr (BASE == 2 || BASE == 4) {
        if (BASE == 2 || !((rodd >> i) & 1u)) {
          const u16x8 r8 = ra[i];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = f32_to_bf16(bf16_to_f32(v[j]) + bf16_to_f32(r8[j]));
        }
      } else if constexpr (EPI == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = bf16_to_f32(v[j]) - e0[j];
          s1[j] += d;
          s2[j] += d * d;
        }
      } else if constexpr (EPI == 3) {
        const u16x8 z8 = ra[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float z = bf16_to_f32(z8[j]);
          const bool on = z * e0[j] + e1[j] > 0.f;
          const float gv = on ? bf16_to_f32(v[j]) : 0.f;
          s1[j] += gv;
          s2[j] += gv * ((z - e2[j]) * e3[j]);
          if (!on) v[j] = 0;
        }
      }
      if constexpr (FOLD) {  // previous block's bn3: ReLU mask from its output bits + reduce sums
        const u16x8 z8 = rz[i];
        v = bf16_keep_where(v, rp[i]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gv = bf16_to_f32(v[j]);
          s1[j] += gv;
          s2[j] += gv * ((bf16_to_f32(z8[j]) - e2[j]) * e3[j]);
        }
      }
      *reinterpret_cast<u16x8*>(p.c + o) = v;
      if constexpr (FOLD_DS) {  // the masked g back into this thread's own tile slots (epilogue_ds)
        *reinterpret_cast<u16x4*>(Cs + rr * CS + cg * 8) = u16x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<u16x4*>(Cs + rr * CS + cg * 8 + 4) = u16x4{v[4], v[5], v[6], v[7]};
      }
    }
  };
  // EPI 9: second pass over the same rows once the first pass's row registers are dead (the
  // register-staged variant sits at the 256-VGPR budget): the downsample BN input rows zd, then
  // sum(g * (zd - mean2) * invstd2) with g read back from the thread's own tile slots
  auto epilogue_ds = [&](int mt) {
    if constexpr (FOLD_DS) {
      float m2[8], i2[8], s3[8];
      load8(p.mean2, nc, m2);
      load8(p.invstd2, nc, i2);
#pragma unroll
      for (int j = 0; j < 8; ++j) s3[j] = s3l[j];
      const int m0 = mt * BM;
      constexpr int HP = NPASS > 1 ? NPASS / 2 : 1;  // rows in flight per half (register budget)
#pragma unroll
      for (int h0 = 0; h0 < NPASS; h0 += HP) {
        u16x8 zd[HP];
#pragma unroll
        for (int i = 0; i < HP; ++i) {
          const int m = min(m0 + r0 + (h0 + i) * RPP, p.M - 1);
          zd[i] = *reinterpret_cast<const u16x8*>(p.aux3 + orow(m) * p.N + nc);
        }
#pragma unroll
        for (int i = 0; i < HP; ++i) {
          const int rr = r0 + (h0 + i) * RPP;
          if (m0 + rr >= p.M) break;
          const u16x4 lo = *reinterpret_cast<const u16x4*>(Cs + rr * CS + cg * 8);
          const u16x4 hi = *reinterpret_cast<const u16x4*>(Cs + rr * CS + cg * 8 + 4);
          const u16x8 gv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
          for (int j = 0; j < 8; ++j) s3[j] += bf16_to_f32(gv[j]) * ((bf16_to_f32(zd[i][j]) - m2[j]) * i2[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s3l[j] = s3[j];
    }
  };
  auto epilogue = [&](int mt) {
    acc_to_lds();
    lds_barrier();
    epilogue_rows(mt);
    epilogue_ds(mt);
  };

  // one step of the (tile, stage) sequence; SF: the free register set (held step q), SN: step q + 1
  int ckt = 0, cti = 0;  // consumer cursor
  auto step = [&](StageRegs<AR, BCH, AR2>& SF, const StageRegs<AR, BCH, AR2>& SN, int q) {
    if (q + 2 < nq) gload(SF);
    compute(q & 1);
    if (++ckt == nk) {  // tile done
      // The epilogue row reads are issued after the accumulators went to LDS: both staging sets
      // are live here, and acc + staging + 2-4 row streams of NPASS rows overran the 256-VGPR
      // budget of 2 waves / SIMD (the folded data-gradient epilogues spilled 150-290 B / lane).
      lds_barrier();    // all waves are done with the stage buffers (the output tile overlaps)
      acc_to_lds();
      epi_load(mg + cti * GM);
      lds_barrier();
      epilogue_rows(mg + cti * GM);
      epilogue_ds(mg + cti * GM);
      zero_acc();
      ckt = 0;
      ++cti;
      lds_barrier();    // output tile read back before step q + 1 is staged over it
    }
    if (q + 1 < nq) swrite(SN, (q + 1) & 1);
    lds_barrier();
  };

  zero_acc();
  if constexpr (PATCH) {
    static_assert(GLDS && !KS1 && !PRO && BM == 128, "patch staging: 3x3 LDS-DMA path");
    if (mg < mtiles) {  // block-uniform
      const int PW = g.W + 2, ohw = g.OH * g.OW;
      // the tile's rows: image part A (rows oh0 - 1 .. ), optional part B (next image, rows -1 .. )
      const int m0 = mg * BM, mlast = min(m0 + BM, p.M) - 1;
      const int img0 = m0 / ohw, oh0 = (m0 - img0 * ohw) / g.OW;
      const int img1 = mlast / ohw, oh1 = (mlast - img1 * ohw) / g.OW;
      const int nA = img1 == img0 ? oh1 - oh0 + 3 : g.OH - oh0 + 2;
      const int R = img1 == img0 ? nA : nA + oh1 + 3;
      constexpr int PLB = patch_bytes<BN>() / 8;  // bytes per 16-B channel plane (fixed: immediates)
      // A-fragment rows of this lane: byte offset of tap (0, 0) in its plane (rows past M: slot 0)
      uint32_t abase[TM];
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0 + wm + 32 * j + fr;
        int sl = 0;
        if (m < p.M) {
          const int im = static_cast<int>(fdiv(static_cast<uint32_t>(m), p.fd_ohw)), r = m - im * ohw,
                    oh = static_cast<int>(fdiv(static_cast<uint32_t>(r), p.fd_ow)), ow = r - oh * g.OW;
          sl = (im == img0 ? oh - oh0 : nA + oh) * PW + ow;
        }
        abase[j] = static_cast<uint32_t>(fh * PLB + sl * 16);  // bytes from the LDS base
      }
      const uint16_t* gb[BI_P];
      const int lrow = lane >> 3, lch = lane & 7;
#pragma unroll
      for (int i = 0; i < BI_P; ++i) {
        const int r = (wave * BI_P + i) * 8 + lrow;
        gb[i] = p.b + static_cast<int64_t>(n0 + r) * p.K + swz(r, lch) * 8;
      }
      auto issue_b = [&](int tap, int cc, int buf) {
        uint16_t* Bs = lds + B_BASE + buf * (BN * kBK);
        const int k0 = tap * g.C + cc * kBK;
#pragma unroll
        for (int i = 0; i < BI_P; ++i)
          __builtin_amdgcn_global_load_lds((gptr_t*)(gb[i] + k0), (lptr_t*)(Bs + (wave * BI_P + i) * 8 * kBK), 16, 0,
                                           0);
      };
      // patch of channel chunk cc: plane pl, piece k of the plane (1 KiB, lane-linear slots); the
      // plane's tail past R x PW slots loads the zero page
      const int nsl = R * PW, ppp = (nsl + 63) / 64, npiece = 8 * ppp;
      auto issue_patch = [&](int cc) {
        for (int pc = wave; pc < npiece; pc += 4) {  // wave-uniform trip count
          const int pl = pc / ppp, sl = (pc - pl * ppp) * 64 + lane, prow = sl / PW, pcol = sl - prow * PW;
          const int im = prow < nA ? img0 : img1, ih = prow < nA ? oh0 - 1 + prow : prow - nA - 1, iw = pcol - 1;
          const bool ok = sl < nsl && static_cast<unsigned>(ih) < static_cast<unsigned>(g.H) &&
                          static_cast<unsigned>(iw) < static_cast<unsigned>(g.W);
          const uint16_t* src =
              ok ? p.a + ((static_cast<int64_t>(im) * g.H + ih) * g.W + iw) * g.C + cc * kBK + pl * 8 : kZeroPage;
          __builtin_amdgcn_global_load_lds((gptr_t*)src,
                                           (lptr_t*)(reinterpret_cast<uint8_t*>(lds) + pl * PLB + (pc - pl * ppp) * 1024),
                                           16, 0, 0);
        }
      };
      auto compute_patch = [&](int buf, int tapoff) {
        const uint16_t* Bs = lds + B_BASE + buf * (BN * kBK);
        uint32_t aa[TM];
#pragma unroll
        for (int j = 0; j < TM; ++j) aa[j] = abase[j] + tapoff * 16;
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int ch = 2 * s2 + fh;
          bf16x8_t xa[TM], wb[TN];
#pragma unroll
          for (int j = 0; j < TM; ++j)
            xa[j] = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const uint8_t*>(lds) + aa[j] + 2 * s2 * PLB);
#pragma unroll
          for (int i = 0; i < TN; ++i) {
            const int r = wn + 32 * i + fr;
            wb[i] = *reinterpret_cast<const bf16x8_t*>(Bs + r * kBK + swz(r, ch) * 8);
          }
#pragma unroll
          for (int i = 0; i < TN; ++i)
#pragma unroll
            for (int j = 0; j < TM; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wb[i], xa[j], acc[i][j], 0, 0, 0);
        }
      };
      const int ncc = g.C / kBK;
      issue_patch(0);
      issue_b(0, 0, 0);
      int st = 0;
      for (int cc = 0; cc < ncc; ++cc) {
        for (int kh = 0; kh < 3; ++kh)
          for (int kw = 0; kw < 3; ++kw, ++st) {
            const int tap = kh * 3 + kw;
            const bool next_same = tap < 8;  // the next stage reuses this patch
            if (next_same) {
              issue_b(tap + 1, cc, (st + 1) & 1);
              if constexpr (BI_P == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
              else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            } else {
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            lds_barrier();  // every wave's stage DMAs (and the patch) landed
            compute_patch(st & 1, kh * PW + kw);
            lds_barrier();  // stage read out before its buffers are refilled
            if (!next_same && cc + 1 < ncc) {  // next channel chunk: new patch + its first weight stage
              issue_patch(cc + 1);
              issue_b(0, cc + 1, (st + 1) & 1);
            }
          }
      }
      epi_load(mg);
      epilogue(mg);
    }
  } else if constexpr (GLDS) {
    // Deep-K tile, one per block: both operands go global -> LDS by LDS-DMA (global_load_lds,
    // 16 B per lane), no staging registers and no ds_write.  One wave instruction fills 8 rows x
    // 128 B lane-linearly, so the chunk swizzle moves to the SOURCE address (linear destination +
    // swizzled source + swizzled read).  Out-of-map taps / rows past M load the zero page.  Two
    // buffers: issue stage t+1, counted vmcnt for stage t, barrier, MFMAs, barrier.
    static_assert(!PRO || XF_GLDS, "LDS-DMA prologues: the in-place LDS pass variants");
    constexpr int AI = BM / 32, BI = BN / 32;  // LDS-DMA instructions per wave per stage
    const int lrow = lane >> 3, lch = lane & 7;
    int64_t gbase[AI];
    int gih[AI], giw[AI];
    unsigned gok = 0;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int r = (wave * AI + i) * 8 + lrow;
      const PixSrc ps = pix_src_fd(mg * BM + r, p.M, g, p.fd_ohw, p.fd_ow);
      gok |= (ps.img >= 0 ? 1u : 0u) << i;
      gih[i] = ps.ih0;
      giw[i] = ps.iw0;
      gbase[i] = ((static_cast<int64_t>(ps.img > 0 ? ps.img : 0) * g.H + ps.ih0) * g.W + ps.iw0) * g.C +
                 swz(r, lch) * 8;
    }
    const uint16_t* gb[BI];
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int r = (wave * BI + i) * 8 + lrow;
      gb[i] = p.b + static_cast<int64_t>(n0 + r) * p.K + swz(r, lch) * 8;
    }
    int qkh = 0, qkw = 0, qcc = 0;
    auto issue = [&](int kt, int buf) {
      uint16_t* As = lds + buf * (BM * kBK);
      uint16_t* Bs = lds + B_BASE + buf * (BN * kBK);
      // the cursor is wave-uniform; readfirstlane lets the compiler keep it (and the tap offset) in
      // SGPRs: one 64-bit VALU add per instruction below
      const int ukh = __builtin_amdgcn_readfirstlane(qkh), ukw = __builtin_amdgcn_readfirstlane(qkw);
      const int toff = __builtin_amdgcn_readfirstlane(KS1 ? qcc : (ukh * g.W + ukw) * g.C + qcc);
      const uint16_t* abase = p.a + toff;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        bool v = (gok >> i) & 1u;
        if constexpr (!KS1) {
          v = v && static_cast<unsigned>(gih[i] + ukh) < static_cast<unsigned>(g.H) &&
              static_cast<unsigned>(giw[i] + ukw) < static_cast<unsigned>(g.W);
        }
        const uint16_t* src = v ? abase + gbase[i] : kZeroPage;
        __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(As + (wave * AI + i) * 8 * kBK), 16, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < BI; ++i)
        __builtin_amdgcn_global_load_lds((gptr_t*)(gb[i] + kt * kBK), (lptr_t*)(Bs + (wave * BI + i) * 8 * kBK),
                                         16, 0, 0);
      qcc += kBK;
      if (qcc == g.C) {
        qcc = 0;
        if (++qkw == (g.ksw ? g.ksw : g.ks)) {
          qkw = 0;
          ++qkh;
        }
      }
    };
    if constexpr (XF_GLDS) {
      // the second source (BN input z / block residual r) of stage kt into the single Z tile
      auto issue_z = [&](int kt) {
        if constexpr (!TWO_GLDS) return;
        const uint16_t* zbase = p.a2 + kt * kBK;
#pragma unroll
        for (int i = 0; i < AI; ++i) {
          const uint16_t* src = ((gok >> i) & 1u) ? zbase + gbase[i] : kZeroPage;
          __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(lds + Z_BASE + (wave * AI + i) * 8 * kBK), 16,
                                           0, 0);
        }
      };
      // one pass over stage kt's A tile: thread t owns LOGICAL chunk t & 7 (fixed channels, one
      // coefficient load per stage) of rows (t >> 3) + 32 i, at physical chunk swz(r, chunk)
      const int lc = t & 7, tr0 = t >> 3;
      const bool store_a = p.aout != nullptr && n0 == 0;
      auto transform = [&](int kt, int buf) {
        uint16_t* As = lds + buf * (BM * kBK);
        const uint16_t* Zs = lds + Z_BASE;
        const int cc = kt * kBK + lc * 8;
        float c0[8], c1[8], c2[8], c3[8];
        if constexpr (ONE_GLDS) {  // BN + ReLU of the previous layer's output
          load8(p.pro, cc, c0);
          load8(p.pro + g.C, cc, c1);
#pragma unroll
          for (int i = 0; i < BM / 32; ++i) {
            const int r = tr0 + 32 * i, m = mg * BM + r;
            const int off = r * kBK + swz(r, lc) * 8;
            u16x8 v = bn_relu8(*reinterpret_cast<const u16x8*>(As + off), c0, c1);
            if (m >= p.M) v = kZero8;
            *reinterpret_cast<u16x8*>(As + off) = v;
          }
          return;
        }
        if constexpr (BWD) {
          load8(p.bwd, cc, c0);
          load8(p.bwd + g.C, cc, c1);
          load8(p.bwd + 2 * g.C, cc, c2);
        } else {
          load8(p.pro, cc, c0);
          load8(p.pro + g.C, cc, c1);
        }
        const bool dual = RESP && p.pro2 != nullptr;  // block-uniform
        if (dual) {
          load8(p.pro2, cc, c2);
          load8(p.pro2 + g.C, cc, c3);
        }
#pragma unroll
        for (int i = 0; i < BM / 32; ++i) {
          const int r = tr0 + 32 * i, m = mg * BM + r;
          const int off = r * kBK + swz(r, lc) * 8;
          u16x8 v = *reinterpret_cast<const u16x8*>(As + off);
          const u16x8 z8 = *reinterpret_cast<const u16x8*>(Zs + off);
          unsigned ob = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if constexpr (BWD) {
              v[j] = f32_to_bf16(c0[j] * bf16_to_f32(v[j]) + c1[j] * bf16_to_f32(z8[j]) + c2[j]);
            } else {  // the same arithmetic as bn_apply_kernel / bn_apply_dual_kernel
              float o = bf16_to_f32(v[j]) * c0[j] + c1[j];
              if (dual) o = o + (bf16_to_f32(z8[j]) * c2[j] + c3[j]);
              else o += bf16_to_f32(z8[j]);
              o = o > 0.f ? o : 0.f;
              ob |= (o > 0.f ? 1u : 0u) << j;
              v[j] = f32_to_bf16(o);
            }
          }
          const bool ok = m < p.M;
          if (!ok) v = kZero8;  // rows past M stay zero (the epilogue sums skip them anyway)
          *reinterpret_cast<u16x8*>(As + off) = v;
          if (store_a && ok) {
            const int64_t e = static_cast<int64_t>(m) * g.C + cc;
            *reinterpret_cast<u16x8*>(p.aout + e) = v;
            if constexpr (RESP) p.abits[e >> 3] = static_cast<uint8_t>(ob);
          }
        }
      };
      if (mg < mtiles) {  // block-uniform
        issue(0, 0);
        issue_z(0);
        for (int kt = 0; kt < nk; ++kt) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          lds_barrier();  // stage kt's A, B and Z landed; every wave is done with stage kt - 1
          if (kt + 1 < nk) issue(kt + 1, (kt + 1) & 1);
          transform(kt, kt & 1);
          lds_barrier();  // the A tile is transformed and Z is free
          if (kt + 1 < nk) issue_z(kt + 1);
          compute(kt & 1);
        }
        lds_barrier();  // the output tile overlays the stage buffers
        epi_load(mg);
        epilogue(mg);
      }
    } else if (mg < mtiles) {  // block-uniform
      issue(0, 0);
      for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) {
          issue(kt + 1, (kt + 1) & 1);
          // this wave's stage-kt DMAs retired (the AI + BI just issued may stay in flight)
          if constexpr (AI + BI == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
          else if constexpr (AI + BI == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        lds_barrier();  // every wave's stage-kt DMAs landed
        compute(kt & 1);
        lds_barrier();  // stage kt read out before stage kt + 2 is issued into its buffer
      }
      // (issuing these reads before the K loop, behind every stage, measured no faster:
      // scripts/probe_dgrad_epi.py)
      epi_load(mg);
      epilogue(mg);
    }
  } else if (nq > 0) {
    set_rows(mg);
    gload(S0);
    swrite(S0, 0);
    if (nq > 1) gload(S1);
    lds_barrier();
  }
  if constexpr (!GLDS) {
    for (int q = 0; q < nq; q += 2) {
      step(S0, S1, q);
      if (q + 1 < nq) step(S1, S0, q + 1);
    }
  }

  if constexpr (EPI == 1 || EPI == 3 || FOLD) {
    float s3[FOLD_DS ? 8 : 1];
    if constexpr (FOLD_DS) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s3[j] = s3l[j];
      lds_barrier();  // every thread has its sum before the reduction scratch overwrites the slots
    }
    // threads with equal cg: lanes l ^ CPR, l ^ 2 CPR, ... of a wave, then the 4 waves via LDS
#pragma unroll
    for (int off = CPR; off < 64; off <<= 1)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += __shfl_xor(s1[j], off, 64);
        s2[j] += __shfl_xor(s2[j], off, 64);
        if constexpr (FOLD_DS) s3[j] += __shfl_xor(s3[j], off, 64);
      }
    float* red = reinterpret_cast<float*>(lds + BM * CS);
    if (lane < CPR) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[wave * BN + cg * 8 + j] = s1[j];
        red[(4 + wave) * BN + cg * 8 + j] = s2[j];
        if constexpr (FOLD_DS) red[(8 + wave) * BN + cg * 8 + j] = s3[j];
      }
    }
    lds_barrier();
    const int64_t PG = p.pgm > 0 ? p.pgm : GM;  // rows per partial slab
    for (int c = t; c < BN; c += 256) {
      p.part[mg * static_cast<int64_t>(p.N) + n0 + c] = (red[c] + red[BN + c]) + (red[2 * BN + c] + red[3 * BN + c]);
      p.part[(PG + mg) * p.N + n0 + c] = (red[4 * BN + c] + red[5 * BN + c]) + (red[6 * BN + c] + red[7 * BN + c]);
      if constexpr (FOLD_DS)
        p.part[(2 * PG + mg) * p.N + n0 + c] =
            (red[8 * BN + c] + red[9 * BN + c]) + (red[10 * BN + c] + red[11 * BN + c]);
    }
  }
}

template <int BM, int BN, int PRO, int EPI, bool KS1, bool GLDS, int VAR = 0>
__global__ __launch_bounds__(256, 2) void conv_fwd_kernel(const ConvGemmArgs p, int GM) {
  conv_fwd_body<BM, BN, PRO, EPI, KS1, GLDS, VAR>(p, GM, xcd_remap(blockIdx.x, gridDim.x));
}

// The four phase GEMMs of a stride-2 3x3 data gradient (conv_dgrad_s2) in ONE grid: blocks
// [start[i], start[i + 1]) run phase order[i], heaviest (2 x 2 taps) first so the 1-tap phase
// fills the tail.  Every range starts at a multiple of 8, so the XCD remap stays local to it.
// Sequential launches left the chip idle in each launch's tail and ran the 1-tap phase (two
// 64-deep stages per tile) alone at its HBM-latency bound.
struct ConvPhaseArgs {
  ConvGemmArgs ph[4];
  int start[5];  // block ranges in launch order
  int order[4];  // phase of each range
  int gm[4];     // pixel tiles of each phase (one tile per block)
};

template <int BN, int EPI>
__global__ __launch_bounds__(256, 2) void conv_dgrad_phases_kernel(const ConvPhaseArgs P) {
  static_assert(EPI == 0 || EPI == 3, "plain store or the ReLU-mask + BN-backward-sums epilogue");
  const int b = blockIdx.x;
  const int i = b >= P.start[3] ? 3 : b >= P.start[2] ? 2 : b >= P.start[1] ? 1 : 0;
  const int ph = P.order[i];
  conv_fwd_body<128, BN, 0, EPI, false, true, 0>(P.ph[ph], P.gm[ph],
                                                 xcd_remap(b - P.start[i], P.start[i + 1] - P.start[i]));
}

// ------------------------------------------------------------------------------ conv_wgrad
// dW tile [n0, n0 + 64 TNO) x [k0, k0 + 64 TKO) over pixels [mb, me): grid = tiles * nsplit
// blocks; logical id -> tile = id % tiles, split = id / tiles, so blocks on one XCD share a
// pixel range (dZ / A rows through L2).  4 waves as 2 x 2; 64-pixel stages, two LDS buffers.
template <int TNO, int TKO, bool PRO, bool GL>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(const ConvWgradArgs p, int rows_per_split) {
  constexpr int BNO = 64 * TNO, BKO = 64 * TKO;
  constexpr int STAGE = kWM * (BNO + BKO);
  constexpr int GCPR = BNO / 8, XCPR = BKO / 8;                 // 16-B chunks per tile row
  constexpr int GIT = kWM * GCPR / 256, XIT = kWM * XCPR / 256;  // chunks per thread per stage
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * STAGE];

  const ConvGeo& g = p.g;
  // wave id through readfirstlane: provably uniform, so LDS-DMA destinations (M0) and other
  // per-wave addresses stay in SGPRs instead of VALU + v_readfirstlane per instruction
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int ntk = p.K / BKO, tiles = (p.N / BNO) * ntk;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles, tile = L - split * tiles;
  const int tn = tile / ntk;
  const int n0 = tn * BNO, k0 = (tile - tn * ntk) * BKO;
  const int tap = k0 / g.C, cc0 = k0 - tap * g.C, kh = tap / g.ks, kw = tap - kh * g.ks;
  const int mb = split * rows_per_split;
  const int me = min(p.M, mb + rows_per_split);
  const int xc = t % XCPR;  // this thread's A chunk column (fixed: 256 % XCPR == 0)
  float psc[8], psh[8];
  if constexpr (PRO) {
    load8(p.pro, cc0 + xc * 8, psc);
    load8(p.pro + g.C, cc0 + xc * 8, psh);
  }
  u16x8 rg[GIT], rx[XIT];
  unsigned xok = 0;
  auto gload = [&](int mc) {
#pragma unroll
    for (int i = 0; i < GIT; ++i) {
      const int id = t + 256 * i, r = id / GCPR, c = id % GCPR;
      const int m = mc + r < me ? mc + r : mb;
      rg[i] = *reinterpret_cast<const u16x8*>(p.dz + static_cast<int64_t>(m) * p.N + n0 + c * 8);
    }
    xok = 0;
#pragma unroll
    for (int i = 0; i < XIT; ++i) {
      const int r = (t + 256 * i) / XCPR;
      const PixSrc s = pix_src_fd(mc + r < me ? mc + r : p.M, p.M, g, p.fd_ohw, p.fd_ow);
      const int64_t o = tap_off(s, kh, kw, cc0 + xc * 8, g);
      xok |= (o >= 0 ? 1u : 0u) << i;
      rx[i] = *reinterpret_cast<const u16x8*>(p.x + (o >= 0 ? o : 0));
    }
  };
  auto swrite = [&](int buf, int mc) {
    uint16_t* Gs = lds + buf * STAGE;
    uint16_t* Xs = Gs + kWM * BNO;
#pragma unroll
    for (int i = 0; i < GIT; ++i) {
      const int id = t + 256 * i, r = id / GCPR, c = id % GCPR;
      *reinterpret_cast<u16x8*>(Gs + tr_off<BNO>(r, c * 8)) = mc + r < me ? rg[i] : kZero8;
    }
#pragma unroll
    for (int i = 0; i < XIT; ++i) {
      const int r = (t + 256 * i) / XCPR;
      u16x8 v = rx[i];
      if constexpr (PRO) v = bn_relu8(v, psc, psh);
      if (!((xok >> i) & 1u)) v = kZero8;
      *reinterpret_cast<u16x8*>(Xs + tr_off<BKO>(r, xc * 8)) = v;
    }
  };

  const int wn = (wave >> 1) * (BNO / 2), wk = (wave & 1) * (BKO / 2);
  f32x16 acc[TNO][TKO];
#pragma unroll
  for (int i = 0; i < TNO; ++i)
#pragma unroll
    for (int j = 0; j < TKO; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  const int nch = me > mb ? (me - mb + kWM - 1) / kWM : 0;  // block-uniform
  auto mma = [&](int buf) {
    const uint16_t* Gs = lds + buf * STAGE;
    const uint16_t* Xs = Gs + kWM * BNO;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8_t ga[TNO], xb[TKO];
#pragma unroll
      for (int i = 0; i < TNO; ++i) ga[i] = tr_frag<BNO>(Gs, s, wn + 32 * i, lane);
#pragma unroll
      for (int j = 0; j < TKO; ++j) xb[j] = tr_frag<BKO>(Xs, s, wk + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < TNO; ++i)
#pragma unroll
        for (int j = 0; j < TKO; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[i], xb[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (GL) {
    // LDS-DMA staging (no prologue): one wave instruction fills 64 consecutive 16-B chunks of
    // the [64][RL] tile, i.e. 1 KB of rows lane-linearly; the transposed-read swizzle moves to
    // the source chunk (tr_off's XOR is an involution).  Rows past the split / out-of-map taps
    // read the zero page.  Two buffers: issue stage ci + 1, counted vmcnt for stage ci.
    static_assert(!PRO, "the BN prologue needs register staging");
    constexpr int GI = GIT, XI = XIT;  // DMA instructions per wave per stage (64 chunks each)
    auto issue = [&](int mc, int buf) {
      uint16_t* Gs = lds + buf * STAGE;
      uint16_t* Xs = Gs + kWM * BNO;
#pragma unroll
      for (int i = 0; i < GI; ++i) {
        const int L = (wave * GI + i) * 64 + lane, r = L / GCPR, pc = L % GCPR;
        const int lc = BNO == 128 ? (pc ^ ((r & 3) << 2)) : (pc ^ (((r >> 1) & 1) << 2));
        const uint16_t* src = mc + r < me ? p.dz + static_cast<int64_t>(mc + r) * p.N + n0 + lc * 8 : kZeroPage;
        __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(Gs + (wave * GI + i) * 512), 16, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int L = (wave * XI + i) * 64 + lane, r = L / XCPR, pc = L % XCPR;
        const int lc = BKO == 128 ? (pc ^ ((r & 3) << 2)) : (pc ^ (((r >> 1) & 1) << 2));
        const PixSrc ps = pix_src_fd(mc + r < me ? mc + r : p.M, p.M, g, p.fd_ohw, p.fd_ow);
        const int64_t o = tap_off(ps, kh, kw, cc0 + lc * 8, g);
        const uint16_t* src = o >= 0 ? p.x + o : kZeroPage;
        __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(Xs + (wave * XI + i) * 512), 16, 0, 0);
      }
    };
    auto mma_gl = [&](int buf) {
      const uint16_t* Gs = lds + buf * STAGE;
      const uint16_t* Xs = Gs + kWM * BNO;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8_t ga[TNO], xb[TKO];
#pragma unroll
        for (int i = 0; i < TNO; ++i) ga[i] = tr_frag_asm<BNO>(Gs, s, wn + 32 * i, lane);
#pragma unroll
        for (int j = 0; j < TKO; ++j) xb[j] = tr_frag_asm<BKO>(Xs, s, wk + 32 * j, lane);
        // the reads landed; the "+v" ties keep every MFMA below the wait
#pragma unroll
        for (int i = 0; i < TNO; ++i) asm volatile("" : "+v"(ga[i]));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < TNO; ++i) asm volatile("" : "+v"(ga[i]));
#pragma unroll
        for (int j = 0; j < TKO; ++j) asm volatile("" : "+v"(xb[j]));
#pragma unroll
        for (int i = 0; i < TNO; ++i)
#pragma unroll
          for (int j = 0; j < TKO; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[i], xb[j], acc[i][j], 0, 0, 0);
      }
    };
    if (nch > 0) {
      issue(mb, 0);
      for (int ci = 0; ci < nch; ++ci) {
        if (ci + 1 < nch) {
          issue(mb + kWM * (ci + 1), (ci + 1) & 1);
          if constexpr (GI + XI == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          else if constexpr (GI + XI == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        lds_barrier();  // every wave's stage-ci DMAs landed
        mma_gl(ci & 1);
        lds_barrier();  // stage ci read out before stage ci + 2 is issued into its buffer
      }
    }
  } else if (nch > 0) {
    gload(mb);
    swrite(0, mb);
    lds_barrier();
    for (int ci = 0; ci < nch; ++ci) {
      const bool more = ci + 1 < nch;
      const int mc = mb + kWM * ci;
      if (more) gload(mc + kWM);
      mma(ci & 1);
      if (more) swrite((ci + 1) & 1, mc + kWM);
      lds_barrier();
    }
  }
  // fp32 slab of this split; register q of lane l: n = .. + (q & 3) + 8 (q >> 2) + 4 (l >> 5),
  // k = .. + (l & 31) -> two 128-B row segments per store instruction
  float* sl = p.ws + static_cast<int64_t>(split) * p.N * p.K;
  const int h = lane >> 5, kl = lane & 31;
#pragma unroll
  for (int i = 0; i < TNO; ++i)
#pragma unroll
    for (int j = 0; j < TKO; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int n = n0 + wn + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
        sl[static_cast<int64_t>(n) * p.K + k0 + wk + 32 * j + kl] = acc[i][j][q];
      }
}

// ------------------------------------------------------------------------------ conv_wgrad (wide)
// The weight gradient is L2-bandwidth bound at 128 x 128 tiles (64 FLOP per staged byte, one
// block round of 2 x 4 waves per CU): this variant runs ONE 8-wave block per CU on a BNO x BKO
// tile of up to 256 x 256 (128 FLOP / byte), WN x WK waves of (32 TN) x (32 TK) each, 32-pixel
// stages through a 4-deep LDS ring filled by LDS-DMA (stage t + 3 in flight while t computes, one
// barrier per stage).  The X tile's 16-B chunks carry their own tap, so a k-tile may span taps
// (3x3 layers with C < BKO).  PRO (1x1 only): the BN + ReLU prologue is applied to the X
// fragments in registers -- a fragment is 8 pixels of ONE channel, so one scale / shift per lane;
// rows past the split read zeros from dz, so their transformed X never contributes.
constexpr int kWP = 32;  // pixels per stage
// LDS ring depth: 3 stages (96 KiB at the 256 x 256 tile) rather than 4 (128 KiB), so smaller
// compute-stream blocks can share a CU with a weight-gradient block running on the side stream:
// ResNet-50 bs1024 +0.4 %, bs256 +0.8 % (2 stages: no further gain; the LDS-pass prologue needs 3,
// its pass runs one stage ahead of the MFMAs -- profiles/r6_wgrad_ring_depth_ab.txt)
constexpr int kWS = 3;
constexpr int kWSP = 3;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 12, "vmcnt immediate");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// PROL (with PRO, 1x1, BKO 128 / 256): the prologue runs as one in-place pass over each staged X
// tile (16 elements per thread per stage) instead of on the X fragments in registers, where each
// of the WN waves sharing a k-column re-transformed it (17-20 VALU per MFMA:
// profiles/r3_resnet50_pmc_ranked_final.txt).
template <int TN, int TK, int WN, int WK, bool PRO, bool DB = false, bool LIN = false, bool PROL = false>
__global__ __launch_bounds__(512, 1) void conv_wgrad_wide_kernel(const ConvWgradArgs p, int rows_per_split) {
  constexpr int BNO = WN * 32 * TN, BKO = WK * 32 * TK;
  static_assert(!PROL || (PRO && (BKO == 128 || BKO == 256)), "LDS-pass prologue: 16-B chunks tile 512 threads");
  static_assert(WN * WK == 8, "8 waves");
  constexpr int WS = PROL ? kWSP : kWS;
  constexpr int STAGE = kWP * (BNO + BKO);
  constexpr int GCPR = BNO / 8, XCPR = BKO / 8;                // 16-B chunks per tile row
  constexpr int GI = kWP * GCPR / 512, XI = kWP * XCPR / 512;  // DMA instructions per wave per stage
  constexpr int PER = GI + XI;
  static_assert(GI >= 1 && XI >= 1 && kWP * GCPR % 512 == 0 && kWP * XCPR % 512 == 0, "tile / stage shape");
  __shared__ __attribute__((aligned(16))) uint16_t lds[WS * STAGE];

  const ConvGeo& g = p.g;
  // wave id through readfirstlane: provably uniform, so LDS-DMA destinations (M0) and other
  // per-wave addresses stay in SGPRs instead of VALU + v_readfirstlane per instruction
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int ntk = p.K / BKO, tiles = (p.N / BNO) * ntk;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles, tile = L - split * tiles;
  const int tn = tile / ntk;
  const int n0 = tn * BNO, k0 = (tile - tn * ntk) * BKO;
  const int mb = split * rows_per_split;
  const int me = min(p.M, mb + rows_per_split);
  const int nst = me > mb ? (me - mb + kWP - 1) / kWP : 0;  // block-uniform

  // per-lane DMA sources: tile row and (swizzled) logical chunk of each instruction
  int grow[GI], gcol[GI], xrow[XI], xkh[XI], xkw[XI], xcc[XI];
#pragma unroll
  for (int i = 0; i < GI; ++i) {
    const int Lc = (wave * GI + i) * 64 + lane, r = Lc / GCPR, pc = Lc % GCPR;
    grow[i] = r;
    gcol[i] = n0 + (pc ^ tr_swz<BNO>(r)) * 8;
  }
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int Lc = (wave * XI + i) * 64 + lane, r = Lc / XCPR, pc = Lc % XCPR;
    const int k = k0 + (pc ^ tr_swz<BKO>(r)) * 8, tap = k / g.C;
    xrow[i] = r;
    xcc[i] = k - tap * g.C;
    xkh[i] = tap / g.ks;
    xkw[i] = tap - xkh[i] * g.ks;
  }
  // Loop-invariant per-lane parts of the DMA sources; a stage adds its (block-uniform, scalar)
  // row base.  1x1 stride-1 pad-0 geometry (every linear layer, most ResNet 1x1 layers): X row m is
  // pixel m, so a source is one 64-bit add -- the general path's two divisions and bounds tests per
  // instruction per stage had made the kernel VALU-bound (~14 VALU per MFMA).
  int64_t goff[GI], xoff[XI];
#pragma unroll
  for (int i = 0; i < GI; ++i) goff[i] = static_cast<int64_t>(grow[i]) * p.N + gcol[i];
#pragma unroll
  for (int i = 0; i < XI; ++i) xoff[i] = static_cast<int64_t>(xrow[i]) * g.C + xcc[i];
  auto issue = [&](int st, int buf) {
    const int mc = mb + st * kWP;
    uint16_t* Gs = lds + buf * STAGE;
    uint16_t* Xs = Gs + kWP * BNO;
    const uint16_t* gb = p.dz + static_cast<int64_t>(mc) * p.N;
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      const uint16_t* src = mc + grow[i] < me ? gb + goff[i] : kZeroPage;
      __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(Gs + (wave * GI + i) * 512), 16, 0, 0);
    }
    if constexpr (LIN) {
      const uint16_t* xb = p.x + static_cast<int64_t>(mc) * g.C;
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const uint16_t* src = mc + xrow[i] < me ? xb + xoff[i] : kZeroPage;
        __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(Xs + (wave * XI + i) * 512), 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int m = mc + xrow[i];
        const PixSrc ps = pix_src_fd(m < me ? m : p.M, p.M, g, p.fd_ohw, p.fd_ow);
        const int64_t o = tap_off(ps, xkh[i], xkw[i], xcc[i], g);
        const uint16_t* src = o >= 0 ? p.x + o : kZeroPage;
        __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(Xs + (wave * XI + i) * 512), 16, 0, 0);
      }
    }
  };

  const int wn = (wave / WK) * (32 * TN), wk = (wave % WK) * (32 * TK);
  float psc[TK], psh[TK];
  if constexpr (PRO) {
#pragma unroll
    for (int j = 0; j < TK; ++j) {
      const int c = (k0 + wk + 32 * j + (lane & 31)) % g.C;
      psc[j] = p.pro[c];
      psh[j] = p.pro[g.C + c];
    }
  }
  f32x16 acc[TN][TK];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  // per-lane fragment addresses (bytes from the stage base), computed once
  uint32_t gfo[TN], xfo[TK];
#pragma unroll
  for (int i = 0; i < TN; ++i) gfo[i] = tr_frag_base<BNO>(wn + 32 * i, lane);
#pragma unroll
  for (int j = 0; j < TK; ++j) xfo[j] = tr_frag_base<BKO>(wk + 32 * j, lane) + kWP * BNO * 2;
  const uint32_t lds_u32 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lptr_t*)lds));
  static_assert(kWP == 32, "two k-steps per stage");
  auto mma = [&](int buf) {
    const uint32_t sb = lds_u32 + static_cast<uint32_t>(buf * STAGE * 2);
    auto kstep = [&](auto SC) {
      constexpr int s = decltype(SC)::value;
      bf16x8_t ga[TN], xb[TK];
#pragma unroll
      for (int i = 0; i < TN; ++i) ga[i] = tr_frag_imm<BNO, s>(sb + gfo[i]);
#pragma unroll
      for (int j = 0; j < TK; ++j) xb[j] = tr_frag_imm<BKO, s>(sb + xfo[j]);
#pragma unroll
      for (int i = 0; i < TN; ++i) asm volatile("" : "+v"(ga[i]));
#pragma unroll
      for (int j = 0; j < TK; ++j) asm volatile("" : "+v"(xb[j]));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < TN; ++i) asm volatile("" : "+v"(ga[i]));
#pragma unroll
      for (int j = 0; j < TK; ++j) asm volatile("" : "+v"(xb[j]));
      if constexpr (PRO && !PROL) {
#pragma unroll
        for (int j = 0; j < TK; ++j) {
          u16x8 v = __builtin_bit_cast(u16x8, xb[j]);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float f = bf16_to_f32(v[e]) * psc[j] + psh[j];
            v[e] = f32_to_bf16(f > 0.f ? f : 0.f);
          }
          xb[j] = __builtin_bit_cast(bf16x8_t, v);
        }
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[i], xb[j], acc[i][j], 0, 0, 0);
    };
    kstep(std::integral_constant<int, 0>{});
    kstep(std::integral_constant<int, 1>{});
  };

  // DB: the blocks of k-tile 0 also sum the staged dz tile's columns (bias gradient): thread t
  // owns 16-B column chunk t % GCPR of rows t / GCPR + (512 / GCPR) i
  const bool dbt = DB && (tile % ntk) == 0;  // block-uniform
  constexpr int DBR = 512 / GCPR;            // threads per column chunk
  float dbacc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // PROL: thread t owns logical X chunk t % XCPR (8 channels, coefficients held in registers) of
  // rows t / XCPR + (512 / XCPR) i -- same swizzle (r & 3) for all of them
  constexpr int XROWS = PROL ? 512 / XCPR : 1, XPT = PROL ? kWP / XROWS : 1;
  float lsc[PROL ? 8 : 1], lsh[PROL ? 8 : 1];
  const int xlc = t % XCPR, xr0 = t / XCPR;
  if constexpr (PROL) {
    load8(p.pro, k0 + xlc * 8, lsc);
    load8(p.pro + g.C, k0 + xlc * 8, lsh);
  }
  auto xform = [&](int buf) {
    if constexpr (PROL) {
      uint16_t* Xs = lds + buf * STAGE + kWP * BNO;
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int r = xr0 + XROWS * i;
        uint16_t* q = Xs + r * BKO + ((xlc ^ tr_swz<BKO>(r)) << 3);
        u16x8 v = *reinterpret_cast<const u16x8*>(q);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = bf16_to_f32(v[e]) * lsc[e] + lsh[e];
          v[e] = f32_to_bf16(f > 0.f ? f : 0.f);
        }
        *reinterpret_cast<u16x8*>(q) = v;
      }
    }
  };
  const int pre = nst < WS - 1 ? nst : WS - 1;
  for (int st = 0; st < pre; ++st) issue(st, st);
  if constexpr (PROL) {
    // the LDS pass runs one stage ahead (stage st + 1 while stage st computes), so the barrier
    // that publishes it is the next iteration's: still one barrier per stage
    if (pre == 3) wait_vmcnt<2 * PER>();
    else if (pre == 2) wait_vmcnt<PER>();
    else wait_vmcnt<0>();
    lds_barrier();
    if (nst > 0) xform(0);
  }
  for (int st = 0; st < nst; ++st) {
    // this wave's DMAs of stage st landed (later stages may stay in flight), then everyone's
    // (PROL: of stage st + 1, whose LDS pass runs in this iteration)
    const int ahead = min(WS - 2, nst - 1 - st);
    if constexpr (PROL) {
      if (ahead >= 2) wait_vmcnt<PER>();
      else wait_vmcnt<0>();
    } else {
      if (ahead >= 2) wait_vmcnt<2 * PER>();
      else if (ahead == 1) wait_vmcnt<PER>();
      else wait_vmcnt<0>();
    }
    lds_barrier();  // also: every wave finished stage st - 1, whose buffer the next issue refills
    if (st + WS - 1 < nst) issue(st + WS - 1, (st + WS - 1) % WS);
    if constexpr (PROL) {
      if (st + 1 < nst) xform((st + 1) % WS);  // published by the next iteration's barrier
    }
    if constexpr (DB) {
      if (dbt) {
        const uint16_t* Gs = lds + (st % WS) * STAGE;
        const int cc = t % GCPR;
#pragma unroll
        for (int r = t / GCPR; r < kWP; r += DBR) {
          const u16x8 v = *reinterpret_cast<const u16x8*>(Gs + r * BNO + ((cc ^ tr_swz<BNO>(r)) << 3));
#pragma unroll
          for (int j = 0; j < 8; ++j) dbacc[j] += bf16_to_f32(v[j]);
        }
      }
    }
    mma(st % WS);
  }
  if constexpr (DB) {
    if (dbt) {
      lds_barrier();  // every wave done with the ring: reuse it for the cross-thread fold
      float* red = reinterpret_cast<float*>(lds);
#pragma unroll
      for (int j = 0; j < 8; ++j) red[t * 8 + j] = dbacc[j];
      lds_barrier();
      if (t < BNO) {
        const int cc = t >> 3, j = t & 7;
        float sum = 0.f;
        for (int k = 0; k < DBR; ++k) sum += red[(k * GCPR + cc) * 8 + j];  // fixed order
        p.dbws[static_cast<int64_t>(split) * p.N + n0 + t] = sum;
      }
    }
  }
  float* sl = p.ws + static_cast<int64_t>(split) * p.N * p.K;
  const int h = lane >> 5, kl = lane & 31;
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int n = n0 + wn + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
        sl[static_cast<int64_t>(n) * p.K + k0 + wk + 32 * j + kl] = acc[i][j][q];
      }
}

// ------------------------------------------------------------------------------ conv_wgrad (patch)
// 3x3 / stride-1 / pad-1 weight gradient at 64-128 channels, where the output dW [N][9C] is small and
// the im2col view re-reads every input pixel once per tap.  A stage is 112 output pixels = R = 112 / W
// whole rows of one image; the block stages the dz rows [112][64 n] and the input PATCH those rows
// touch -- (R + 2) x (W + 2) pixel slots x 64 channels, halo slots zero (out-of-map rows / columns
// load the zero page) -- ONCE, and all nine taps read their B fragments from it at a shifted slot
// (slot(m) + kh (W + 2) + kw): L2 -> LDS traffic per stage drops from 9 x 112 x 64 to
// (R + 2)(W + 2) x 64 pixel-channels.
// LDS layout: both tiles are split into two 32-channel PLANES of 64-B rows (dz: [n half][pixel][32],
// patch: [c half][slot][32]).  A wave reads one plane, and the 4 rows of a ds_read_b64_tr_b16 lane
// group are 4 consecutive pixels (slots) = 256 contiguous bytes = every bank once -- no swizzle, so
// every fragment address is linear: a tap's kw and a k-step's pixel offset become instruction
// immediates and the whole loop runs on 1 + 14 loop-invariant address registers (W % 4 == 0: a
// 4-pixel group never straddles an output row).
// Stride 2 (S = 2): the stage's R output rows touch 2R + 1 input rows; the patch columns are stored
// split by parity ([column parity][row][column / 2]), so tap kw reads parity kw & 1 at column
// ow + kw / 2 -- 4 consecutive output pixels are again 4 consecutive 64-B rows, and kw is again an
// immediate (a two-stage ring: the 2x-wide patch fills the LDS).
// 12 waves: (kh, n half, c half) -> 32 n x 3 taps x 32 c each, one dz fragment + three patch
// fragments per three MFMAs.  Block = (n tile 64, c tile 64, pixel split); fp32 per-split slabs,
// fixed-order reduction (deterministic) as the other weight-gradient kernels.
constexpr int kPP = 112;  // pixels per stage

template <int OFF>
__device__ __forceinline__ s16x4 ds_tr_off(uint32_t a) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF) : "memory");
  return v;
}

template <int W, int S>
__global__ __launch_bounds__(768, 1) void conv_wgrad_patch_kernel(const ConvWgradArgs p, int stages_per_split) {
  constexpr int OW = W / S, R = kPP / OW, PR = S * (R - 1) + 3;  // output rows / input rows per stage
  constexpr int PW = S == 1 ? W + 2 : (W + 2) / 2;            // slots per patch row (per column parity)
  constexpr int KPS = S == 1 ? 3 : 2;                         // LDS ring depth
  static_assert(kPP % OW == 0 && OW % 4 == 0 && W % S == 0, "a stage is whole rows; 4-pixel groups stay in a row");
  constexpr int GPL = kPP * 64;                         // dz plane bytes (32 n per row)
  constexpr int GB = 2 * GPL;                           // dz tile bytes
  constexpr int PPL = S * PR * PW * 64;                 // patch plane bytes
  constexpr int PB = ((2 * PPL + 1023) / 1024) * 1024;  // patch tile bytes (whole 1 KiB DMA pieces)
  constexpr int GI = GB / 1024, PI = PB / 1024;         // DMA pieces
  constexpr int NI = GI + PI;                           // per stage, dealt over the 12 waves
  constexpr int STB = GB + PB;                          // stage bytes
  constexpr int MAXW = (NI + 11) / 12;                  // pieces of the busiest wave
  static_assert(GB % 1024 == 0 && MAXW <= 8 && (KPS == 2 || MAXW <= 4) && KPS * STB <= 160 * 1024, "stage shape");
  __shared__ __attribute__((aligned(16))) uint16_t lds[KPS * STB / 2];

  const ConvGeo& g = p.g;
  // wave id through readfirstlane: provably uniform, so LDS-DMA destinations (M0) and other
  // per-wave addresses stay in SGPRs instead of VALU + v_readfirstlane per instruction
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nct = g.C / 64, tiles = (p.N / 64) * nct;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles, tile = L - split * tiles;
  const int n0 = (tile / nct) * 64, c0 = (tile % nct) * 64;
  const int rows_per_img = g.OH / R, total = p.M / kPP;
  const int sb = split * stages_per_split;
  const int se = min(total, sb + stages_per_split);
  const int nst = se > sb ? se - sb : 0;  // block-uniform

  // ---- DMA: piece i = wave + 12 j (dz pieces first, then patch pieces); lane-linear 16-B chunks,
  // chunk ch of a plane = row ch / 4, 8 channels (ch % 4); sources recomputed per stage
  const int myn = (NI - wave + 11) / 12;  // wave-uniform: MAXW or MAXW - 1
  auto issue = [&](int st, int buf) {
    const int q = sb + st, img = q / rows_per_img, ih0 = (q - img * rows_per_img) * R * S - 1;
    uint8_t* base = reinterpret_cast<uint8_t*>(lds) + buf * STB;
    const uint16_t* gsrc = p.dz + static_cast<int64_t>(q) * kPP * p.N + n0;
    const uint16_t* xsrc = p.x + (static_cast<int64_t>(img) * g.H + ih0) * g.W * g.C + c0;
#pragma unroll
    for (int j = 0; j < MAXW; ++j) {
      if (j >= myn) break;  // wave-uniform
      const int i = wave + 12 * j;
      const uint16_t* src;
      if (i < GI) {  // wave-uniform
        const int ch = i * 64 + lane, pl = ch / (GPL / 16), r = ch - pl * (GPL / 16);
        src = gsrc + static_cast<int64_t>(r >> 2) * p.N + pl * 32 + (r & 3) * 8;
      } else {  // slot (parity, pr, j): input pixel (ih0 + pr, S j + parity - 1); halo / out-of-map: zero
        const int ch = (i - GI) * 64 + lane, pl = ch / (PPL / 16), r = ch - pl * (PPL / 16), slot = r >> 2;
        const int par = slot / (PR * PW), rem = slot - par * (PR * PW), pr = rem / PW;
        const int pc = S * (rem - pr * PW) + par, ih = ih0 + pr;
        const bool ok = pl < 2 && pc >= 1 && pc <= W && static_cast<unsigned>(ih) < static_cast<unsigned>(g.H);
        src = ok ? xsrc + (static_cast<int64_t>(pr) * W + (pc - 1)) * g.C + pl * 32 + (r & 3) * 8 : kZeroPage;
      }
      __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(base + i * 1024), 16, 0, 0);
    }
  };

  // ---- fragment addresses (bytes inside a stage): lane reads pixel m = 16 s + 4 h + mrow, columns
  // 16 (gi & 1) + 4 (i16 & 3) .. + 3 of its plane; s / h / kw are immediates except the patch slot
  const int kh = wave % 3, nh = (wave / 3) & 1, chf = wave / 6;
  const int gi = lane >> 4, i16 = lane & 15;
  const int mrow = 8 * (gi >> 1) + (i16 >> 2), colb = (16 * (gi & 1) + 4 * (i16 & 3)) * 2;
  const uint32_t ga = static_cast<uint32_t>(nh * GPL + mrow * 64 + colb);
  uint32_t xa[7][2];
#pragma unroll
  for (int s = 0; s < 7; ++s)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = 16 * s + 4 * h + mrow, oh = m / OW, ow = m - oh * OW;
      xa[s][h] = static_cast<uint32_t>(GB + chf * PPL + ((S * oh + kh) * PW + ow) * 64 + colb);
    }

  f32x16 acc[3];
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[k][q] = 0.f;
  auto mma = [&](int buf) {
    const uint32_t b0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const lds_s16x4*)lds)) + buf * STB;
    const uint32_t gb = b0 + ga;
    // byte offsets of taps kw = 1, 2 from kw = 0: the next slot (stride 1); the odd-column parity
    // block / the next even slot (stride 2)
    constexpr int K1 = S == 1 ? 64 : PR * PW * 64, K2 = S == 1 ? 128 : 64;
#define PSAMD_PATCH_STEP(Q)                                                                              \
  {                                                                                                      \
    s16x4 a0 = ds_tr_off<(16 * Q) * 64>(gb), a1 = ds_tr_off<(16 * Q + 4) * 64>(gb);                      \
    const uint32_t x0 = b0 + xa[Q][0], x1 = b0 + xa[Q][1];                                               \
    s16x4 p00 = ds_tr_off<0>(x0), p01 = ds_tr_off<0>(x1);                                                \
    s16x4 p10 = ds_tr_off<K1>(x0), p11 = ds_tr_off<K1>(x1);                                              \
    s16x4 p20 = ds_tr_off<K2>(x0), p21 = ds_tr_off<K2>(x1);                                              \
    /* the reads land asynchronously: the wait redefines their registers, so no MFMA is scheduled  */   \
    /* above it and no register is reused before it                                               */   \
    asm volatile("s_waitcnt lgkmcnt(0)"                                                                  \
                 : "+v"(a0), "+v"(a1), "+v"(p00), "+v"(p01), "+v"(p10), "+v"(p11), "+v"(p20), "+v"(p21)  \
                 :                                                                                       \
                 : "memory");                                                                            \
    const bf16x8_t af = as_bf16x8(s16x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]});        \
    acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(                                                    \
        af, as_bf16x8(s16x8{p00[0], p00[1], p00[2], p00[3], p01[0], p01[1], p01[2], p01[3]}), acc[0], 0, 0, 0); \
    acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(                                                    \
        af, as_bf16x8(s16x8{p10[0], p10[1], p10[2], p10[3], p11[0], p11[1], p11[2], p11[3]}), acc[1], 0, 0, 0); \
    acc[2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(                                                    \
        af, as_bf16x8(s16x8{p20[0], p20[1], p20[2], p20[3], p21[0], p21[1], p21[2], p21[3]}), acc[2], 0, 0, 0); \
  }
    PSAMD_PATCH_STEP(0)
    PSAMD_PATCH_STEP(1)
    PSAMD_PATCH_STEP(2)
    PSAMD_PATCH_STEP(3)
    PSAMD_PATCH_STEP(4)
    PSAMD_PATCH_STEP(5)
    PSAMD_PATCH_STEP(6)
#undef PSAMD_PATCH_STEP
  };

  const int pre = nst < KPS - 1 ? nst : KPS - 1;
  for (int st = 0; st < pre; ++st) issue(st, st);
  for (int st = 0; st < nst; ++st) {
    // this wave's DMAs of stage st landed (the next stage's may stay in flight), then everyone's
    if (KPS == 3 && st + 1 < nst) {
      if (myn == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (myn == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if (myn == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();  // also: every wave finished stage st - 1, whose buffer the next issue refills
    if (st + KPS - 1 < nst) issue(st + KPS - 1, (st + KPS - 1) % KPS);
    mma(st % KPS);
  }
  // slab[split][n][k], k = (kh * 3 + kw) * C + c
  float* sl = p.ws + static_cast<int64_t>(split) * p.N * p.K;
  const int h = lane >> 5, cl = lane & 31;
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int n = n0 + nh * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
      const int k = (kh * 3 + kw) * g.C + c0 + chf * 32 + cl;
      sl[static_cast<int64_t>(n) * p.K + k] = acc[kw][q];
    }
}

// out[y][e] = sum_{b in [y*per, y*per + per)} in[b][e] in fixed order (bf16 or fp32 out)
template <bool BF16>
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ in, int nslab, int per, int64_t E,
                                                          void* __restrict__ out) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= E) return;
  const int b0 = blockIdx.y * per, b1 = min(nslab, b0 + per);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int b = b0;
  for (; b + 3 < b1; b += 4) {
    a0 += in[b * E + e];
    a1 += in[(b + 1) * E + e];
    a2 += in[(b + 2) * E + e];
    a3 += in[(b + 3) * E + e];
  }
  for (; b < b1; ++b) a0 += in[b * E + e];
  const float v = (a0 + a1) + (a2 + a3);
  if constexpr (BF16) static_cast<uint16_t*>(out)[blockIdx.y * E + e] = f32_to_bf16(v);
  else static_cast<float*>(out)[blockIdx.y * E + e] = v;
}

// ------------------------------------------------------------------------------ weight_prep
// The data-gradient GEMMs read every bottleneck weight in a second layout: the 1x1 weights
// transposed, the stride-1 3x3 weight flipped and channel-transposed, the stride-2 3x3 weight
// gathered into its four phase matrices.  Built per weight these were ~70 tiny copy / flip /
// gather kernels per ResNet-50 step (0.64 ms); here ONE launch builds all of them, one job per
// blockIdx.y, at the start of the forward (the weights are final for the step by then).
// Destination-major iteration: coalesced writes, gathered reads (every weight is L2-resident).
struct WPrepJob {
  const uint16_t* src;  // channels_last weight [A][ks][ks][B] (A = output channels, B = input)
  uint16_t* dst;
  int kind;             // 0: 1x1 [A][B] -> [B][A]; 1: 3x3 -> [B][3][3][A] flipped; 2: 3x3 -> 4 phases
  int A, B;
};

// Every layout is a set of 2D transposes (a 1x1 weight: one; a 3x3: one per tap, nine in all for
// the flipped layout and for the four stride-2 phases together): source rows r (A of them, the
// weight's first index) with the channel c contiguous, destination rows c with r contiguous.
// One block moves one 64 x 64 tile of one of them through LDS, so both the reads and the writes
// are coalesced (the element-per-thread gather with 64-bit index divisions took 0.16-0.18 ms per
// step for 51 MB; profiles/r4_resnet50_step_breakdown_baseline.txt).
__global__ __launch_bounds__(256) void weight_prep_kernel(const WPrepJob* __restrict__ jobs) {
  const WPrepJob jb = jobs[blockIdx.y];
  const int A = jb.A, B = jb.B, ta = (A + 63) / 64, tb = (B + 63) / 64, tiles = ta * tb;
  const int nsub = jb.kind == 0 ? 1 : 9;
  const int idx = blockIdx.x;
  if (idx >= nsub * tiles) return;  // block-uniform
  const int sub = idx / tiles, ti = idx - sub * tiles, r0 = (ti / tb) * 64, c0 = (ti - (ti / tb) * tb) * 64;
  int64_t soff = 0, ss = B, doff = 0, ds = A;
  if (jb.kind == 1) {  // dst[c][kh][kw][r] = src[r][2 - kh][2 - kw][c]
    const int kh = sub / 3, kw = sub - kh * 3;
    soff = ((2 - kh) * 3 + (2 - kw)) * static_cast<int64_t>(B);
    ss = 9 * static_cast<int64_t>(B);
    doff = sub * static_cast<int64_t>(A);
    ds = 9 * static_cast<int64_t>(A);
  } else if (jb.kind == 2) {
    // phases (0,0) (0,1) (1,0) (1,1) at 0, AB, 3AB, 5AB, each [B][nh][nw][A]; sub -> (phase, dh, dw)
    const int ph = sub == 0 ? 0 : sub < 3 ? 1 : sub < 5 ? 2 : 3;
    const int q = sub - (ph == 0 ? 0 : ph == 1 ? 1 : ph == 2 ? 3 : 5);
    const int pa = ph >> 1, pb = ph & 1, nh = pa ? 2 : 1, nw = pb ? 2 : 1;
    const int dh = q / nw, dw = q - dh * nw;
    const int kh = pa ? (dh ? 0 : 2) : 1, kw = pb ? (dw ? 0 : 2) : 1;
    const int64_t AB = static_cast<int64_t>(A) * B;
    soff = (kh * 3 + kw) * static_cast<int64_t>(B);
    ss = 9 * static_cast<int64_t>(B);
    doff = (ph == 0 ? 0 : ph == 1 ? AB : ph == 2 ? 3 * AB : 5 * AB) + (dh * nw + dw) * static_cast<int64_t>(A);
    ds = static_cast<int64_t>(nh) * nw * A;
  }
  __shared__ uint16_t tile[64][66];
  const int t = threadIdx.x, tc = t & 63, tr = t >> 6;
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int r = r0 + tr + 4 * i, c = c0 + tc;
    if (r < A && c < B) tile[tr + 4 * i][tc] = jb.src[soff + r * ss + c];
  }
  __syncthreads();
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int c = c0 + tr + 4 * i, r = r0 + tc;
    if (r < A && c < B) jb.dst[doff + c * ds + r] = tile[tc][tr + 4 * i];
  }
}

void launch_weight_prep(const void* jobs, int njobs, int max_blocks, hipStream_t s) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(weight_prep_kernel, dim3(max_blocks, njobs), dim3(256), 0, s, static_cast<const WPrepJob*>(jobs));
}

// ------------------------------------------------------------------------------ launchers
// Forward tile plan.  HBM-bound shallow-K layers (<= 2 stages; <= 4 with the BN prologue, whose
// register staging gains most from the cross-tile prefetch: scripts/probe_conv_fwd.py) run a
// persistent grid of 2 blocks per CU (statistics kept in registers); deeper K runs one block per
// tile so the hardware balances the tail.
constexpr int kPersistNkPro = 4;  // 4-stage PRO layers: cross-tile prefetch pays (L3 conv3 -8%)

// 3x3 / stride 1 / pad 1 forward (or data gradient) whose 128-pixel tiles' patch fits the LDS
// budget and spans at most two images
bool patch_fwd_ok(const ConvGeo& g, int N, bool pro) {
  if (pro || g.ks != 3 || (g.ksw != 0 && g.ksw != 3) || g.stride != 1 || g.pad != 1 ||
      g.RH != 0 || g.OH != g.H || g.OW != g.W || g.C % 64 != 0 || g.OH * g.OW < 128)
    return false;
  // 64-channel outputs keep the tall 256 x 64 im2col tile: the 128 x 64 patch tile (64 x 32 per
  // wave, 1.5 fragment reads per MFMA) measured 9-14 % slower there (profiles/r3_conv_patch_fwd_ab.txt)
  if (N % 128 != 0) return false;
  const int bn = N % 128 == 0 ? 128 : 64;
  const int span = (g.OW - 1 + 128 + g.OW - 1) / g.OW, rmax = span + 4;
  const int plane = (rmax * (g.W + 2) * 16 + 1023) / 1024 * 1024;  // one 16-B channel plane, whole pieces
  return 8 * plane <= (bn == 64 ? patch_bytes<64>() : patch_bytes<128>());
}

// two-source prologues with K >= 64 x this run on the LDS-DMA variant (profiles/r4_twosrc_probe.txt:
// LDS-DMA ahead at every K >= 256)
constexpr int kTwosrcGldsMinNk = 4;

// src2: two-source prologue of the launch (0 none, 1 block output, 2 BN backward)
bool twosrc_glds(int K, int src2) { return src2 != 0 && K / kBK >= kTwosrcGldsMinNk; }

ConvFwdPlan conv_fwd_plan_geo(int M, int N, int K, bool pro, const ConvGeo& g, int src2, int epi) {
  if (const int tn = conv_big_tn(M, N, K, pro, g, src2, epi)) {  // 256 x TN tiles (conv_big.hip)
    ConvFwdPlan pl;
    pl.bm = 256;
    pl.bn = tn;
    pl.gm = conv_big_gm(M);
    return pl;
  }
  if (twosrc_glds(K, src2)) {  // LDS-DMA two-source prologue: one 128-pixel tile per block
    ConvFwdPlan pl;
    pl.bm = 128;
    pl.bn = N % 128 == 0 ? 128 : 64;
    pl.gm = (M + 127) / 128;
    return pl;
  }
  if (src2 == 1) {  // block-output prologue: 64-channel tiles (128 x 128 with two row sources spilled)
    ConvFwdPlan pl = conv_fwd_plan(M, N, K, true);
    pl.bn = 64;
    if (pl.gm != (M + 127) / 128) pl.gm = std::max(1, std::min((M + 127) / 128, 512 / (N / 64)));
    return pl;
  }
  if (patch_fwd_ok(g, N, pro)) {  // one 128-pixel tile per block (LDS-DMA path)
    ConvFwdPlan pl;
    pl.bm = 128;
    pl.bn = N % 128 == 0 ? 128 : 64;
    pl.gm = (M + 127) / 128;
    return pl;
  }
  return conv_fwd_plan(M, N, K, pro, epi);
}

ConvFwdPlan conv_fwd_plan(int M, int N, int K, bool pro, int epi) {
  ConvFwdPlan pl;
  if (!pro && N == 64 && K / kBK >= 8) {  // 64-channel 3x3 (K = 576): 256 x 64 tiles
    pl.bm = 256;
    pl.bn = 64;
    pl.gm = (M + 255) / 256;
    return pl;
  }
  pl.bn = N % 128 == 0 ? 128 : 64;
  const int nN = N / pl.bn;
  pl.bm = 128;  // (64-pixel tiles measured slower on every ResNet-50 shape: scripts/probe_convgemm.py)
  const int nk = K / kBK;
  // (a persistent grid for the read-heavy data-gradient epilogues measured no faster at 4-16
  // stages: scripts/probe_dgrad_epi.py)
  const bool persist = nk <= 2 || (pro && nk <= kPersistNkPro);
  pl.gm = !persist ? (M + 127) / 128 : std::max(1, std::min((M + 127) / 128, 512 / nN));
  return pl;
}

void launch_conv_fwd(const ConvGemmArgs& a0, hipStream_t s) {
  if (a0.M <= 0) return;
  ConvGemmArgs a = a0;
  a.fd_ohw = make_fastdiv(static_cast<uint32_t>(a.g.OH * a.g.OW));
  a.fd_ow = make_fastdiv(static_cast<uint32_t>(a.g.OW));
  const bool bwd = a.bwd != nullptr;
  const bool resp = a.pro != nullptr && a.a2 != nullptr && !bwd;
  const int src2 = resp ? 1 : bwd ? 2 : 0;
  const ConvFwdPlan pl = conv_fwd_plan_geo(a.M, a.N, a.K, a.pro != nullptr || bwd, a.g, src2, a.epi);
  const int GM = pl.gm;
  const int nblk = GM * (a.N / pl.bn);
  if (conv_big_ok(a.M, a.N, a.K, a.pro != nullptr || bwd, a.g, src2, a.epi)) {
    launch_conv_big(a, s);
    return;
  }
  if (twosrc_glds(a.K, src2)) {  // (1x1: the binding checks)
#define PSAMD_CF2S(BN, PRO, EPI) \
  hipLaunchKernelGGL((conv_fwd_kernel<128, BN, PRO, EPI, true, true>), dim3(nblk), dim3(256), 0, s, a, GM)
    if (resp) {
      if (pl.bn == 128) {
        if (a.epi == 1) { PSAMD_CF2S(128, 3, 1); } else { PSAMD_CF2S(128, 3, 0); }
      } else {
        if (a.epi == 1) { PSAMD_CF2S(64, 3, 1); } else { PSAMD_CF2S(64, 3, 0); }
      }
    } else {
      if (pl.bn == 128) { PSAMD_CF2S(128, 2, 3); } else { PSAMD_CF2S(64, 2, 3); }
    }
#undef PSAMD_CF2S
    return;
  }
  if (!bwd && patch_fwd_ok(a.g, a.N, a.pro != nullptr) && (a.epi == 0 || a.epi == 1 || a.epi == 3)) {
#define PSAMD_CFP(BN, EPI) \
  hipLaunchKernelGGL((conv_fwd_kernel<128, BN, 0, EPI, false, true, true>), dim3(nblk), dim3(256), 0, s, a, GM)
    if (pl.bn == 128) {
      if (a.epi == 1) { PSAMD_CFP(128, 1); } else if (a.epi == 3) { PSAMD_CFP(128, 3); } else { PSAMD_CFP(128, 0); }
    } else {
      if (a.epi == 1) { PSAMD_CFP(64, 1); } else if (a.epi == 3) { PSAMD_CFP(64, 3); } else { PSAMD_CFP(64, 0); }
    }
#undef PSAMD_CFP
    return;
  }
  const bool ks1 = a.g.ks == 1 && a.g.ksw <= 1;
  // deep K without the BN prologue: LDS-DMA staging (one tile per block)
  const bool glds = !a.pro && !bwd && pl.gm == (a.M + pl.bm - 1) / pl.bm && a.K / kBK > 2;
#define PSAMD_CF3(BM, BN, PRO, EPI, GL)                                                                          \
  if (ks1) hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, PRO, EPI, true, GL>), dim3(nblk), dim3(256), 0, s, a, GM); \
  else hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, PRO, EPI, false, GL>), dim3(nblk), dim3(256), 0, s, a, GM)
#define PSAMD_CF2(BM, BN, PRO, EPI)                        \
  if constexpr (PRO) { PSAMD_CF3(BM, BN, PRO, EPI, false); } \
  else if (glds) { PSAMD_CF3(BM, BN, PRO, EPI, true); }       \
  else { PSAMD_CF3(BM, BN, PRO, EPI, false); }
#define PSAMD_CF(BN, PRO, EPI) PSAMD_CF2(128, BN, PRO, EPI)
#define PSAMD_CFE(BN, PRO)               \
  switch (a.epi) {                       \
    case 1: PSAMD_CF(BN, PRO, 1); break; \
    case 2: PSAMD_CF(BN, PRO, 2); break; \
    case 3: PSAMD_CF(BN, PRO, 3); break; \
    case 4: PSAMD_CF(BN, PRO, 4); break; \
    case 5: PSAMD_CF(BN, PRO, 5); break; \
    case 6: PSAMD_CF(BN, PRO, 6); break; \
    case 7: PSAMD_CF(BN, PRO, 7); break; \
    case 8: PSAMD_CF(BN, PRO, 8); break; \
    case 9: PSAMD_CF(BN, PRO, 9); break; \
    default: PSAMD_CF(BN, PRO, 0); break; \
  }
  if (pl.bm == 256) {  // LDS-DMA only (no prologue, deep K)
#define PSAMD_CFT(EPI) PSAMD_CF3(256, 64, false, EPI, true)
    switch (a.epi) {
      case 1: PSAMD_CFT(1); break;
      case 2: PSAMD_CFT(2); break;
      case 3: PSAMD_CFT(3); break;
      case 4: PSAMD_CFT(4); break;
      case 5: PSAMD_CFT(5); break;
      case 6: PSAMD_CFT(6); break;
      case 7: PSAMD_CFT(7); break;
      case 8: PSAMD_CFT(8); break;
      default: PSAMD_CFT(0); break;
    }
#undef PSAMD_CFT
    return;
  }
  if (resp) {  // 1x1 forward over the previous block's output, applied while staging
#define PSAMD_CFR(BN, EPI) \
  hipLaunchKernelGGL((conv_fwd_kernel<128, BN, 3, EPI, true, false>), dim3(nblk), dim3(256), 0, s, a, GM)
    if (pl.bn == 128) {
      if (a.epi == 1) { PSAMD_CFR(128, 1); } else { PSAMD_CFR(128, 0); }
    } else {
      if (a.epi == 1) { PSAMD_CFR(64, 1); } else { PSAMD_CFR(64, 0); }
    }
#undef PSAMD_CFR
    return;
  }
  if (bwd) {  // 1x1 data gradient with the previous BN's backward in the prologue (epilogue 3)
    if (pl.bn == 128) hipLaunchKernelGGL((conv_fwd_kernel<128, 128, 2, 3, true, false>), dim3(nblk), dim3(256), 0, s, a, GM);
    else hipLaunchKernelGGL((conv_fwd_kernel<128, 64, 2, 3, true, false>), dim3(nblk), dim3(256), 0, s, a, GM);
    return;
  }
  // the BN prologue only appears on forward convolutions (epilogue 0 / 1)
  if (pl.bn == 128) {
    if (a.pro) {
      if (a.epi == 1) { PSAMD_CF(128, true, 1); } else { PSAMD_CF(128, true, 0); }
    } else { PSAMD_CFE(128, false) }
  } else {
    if (a.pro) {
      if (a.epi == 1) { PSAMD_CF(64, true, 1); } else { PSAMD_CF(64, true, 0); }
    } else { PSAMD_CFE(64, false) }
  }
#undef PSAMD_CFE
#undef PSAMD_CF
#undef PSAMD_CF2
#undef PSAMD_CF3
}

int conv_dgrad_phase_gm(int M) { return (M + 127) / 128; }

void launch_conv_dgrad_phases(const ConvGemmArgs* ph, hipStream_t s) {
  ConvPhaseArgs P{};
  const int N = ph[0].N;
  const int bn = N % 128 == 0 ? 128 : 64;
  static constexpr int kOrder[4] = {3, 1, 2, 0};  // taps 4, 2, 2, 1
  int at = 0;
  for (int i = 0; i < 4; ++i) {
    const int q = kOrder[i];
    P.ph[q] = ph[q];
    P.ph[q].fd_ohw = make_fastdiv(static_cast<uint32_t>(ph[q].g.OH * ph[q].g.OW));
    P.ph[q].fd_ow = make_fastdiv(static_cast<uint32_t>(ph[q].g.OW));
    P.gm[q] = conv_dgrad_phase_gm(ph[q].M);
    P.order[i] = q;
    P.start[i] = at;
    at += (P.gm[q] * (N / bn) + 7) / 8 * 8;  // ranges start at multiples of 8 (XCD-local remap)
  }
  P.start[4] = at;
  if (at == 0) return;
  const bool e3 = ph[0].epi == 3;  // (the binding allows 0 or 3 and sets the part / aux / mc of epi 3)
  if (bn == 128) {
    if (e3) hipLaunchKernelGGL((conv_dgrad_phases_kernel<128, 3>), dim3(at), dim3(256), 0, s, P);
    else hipLaunchKernelGGL((conv_dgrad_phases_kernel<128, 0>), dim3(at), dim3(256), 0, s, P);
  } else {
    if (e3) hipLaunchKernelGGL((conv_dgrad_phases_kernel<64, 3>), dim3(at), dim3(256), 0, s, P);
    else hipLaunchKernelGGL((conv_dgrad_phases_kernel<64, 0>), dim3(at), dim3(256), 0, s, P);
  }
}

namespace {
struct WPlan {
  int tno, tko, tiles, nsplit, rows, groups;
  int wide;  // 0: conv_wgrad_kernel; wide tiles 1: 256 x 256, 2: 256 x 128, 3: 128 x 256, 4: 128 x 384
};

// Slab reduction levels: > 16 slabs reduce in two fixed-order levels (16 slabs per first-level
// group) unless the weight has >= 256K elements -- then one thread per element over every slab
// already fills the chip, and the second launch (plus its gap) is saved.
int slab_groups(int nsplit, int64_t E) {
  if (nsplit <= 16 || (E >= (int64_t(1) << 18) && nsplit <= 64)) return 0;
  return (nsplit + 15) / 16;
}

// Split count that fills WHOLE rounds of `slots` resident blocks (one or two rounds), at most
// `cap` splits: rounding the block count up past a round (e.g. 9 tiles x 57 splits = 513 of 512)
// adds a round of one block and halves the kernel's throughput.
int fill_rounds(int tiles, int slots, int cap) {
  int ns = 1;
  double best = -1.0;
  for (int rounds = 1; rounds <= 2; ++rounds) {
    const int cand = std::max(1, std::min(rounds * slots / tiles, cap));
    const int blocks = cand * tiles;
    const double eff = static_cast<double>(blocks) / (((blocks + slots - 1) / slots) * static_cast<double>(slots));
    if (eff > best + 0.02) {
      best = eff;
      ns = cand;
    }
  }
  return ns;
}

// Wide tiles (one 8-wave block per CU) where N and K allow a 256-wide side and the prologue, if
// any, is on a 1x1 layer; else 64 / 128 tiles (a k-tile must not straddle taps), 2 blocks per CU.
// >= 4 (8 for wide) stages per split; > 16 slabs reduce in two fixed-order levels.
WPlan wplan(int M, int N, int K, int C, bool pro) {
  WPlan w{};
  const bool ks1 = K == C;
  int bno = N % 256 == 0 ? 256 : 128, bko = K % 256 == 0 ? 256 : 128;
  if (bno == 128 && bko == 128 && K % 384 == 0) bko = 384;  // 3x3 at C = 128: 3 taps per k-tile
  if ((!pro || ks1) && N % 128 == 0 && K % 128 == 0 && C % 8 == 0 && (bno == 256 || bko > 128)) {
    w.wide = bno == 256 ? (bko == 256 ? 1 : 2) : bko == 256 ? 3 : 4;
    w.tiles = (N / bno) * (K / bko);
    const int chunks = (M + kWP - 1) / kWP;
    const int ns = fill_rounds(w.tiles, 256, std::max(1, chunks / 8));
    w.rows = ((chunks + ns - 1) / ns) * kWP;
  } else {
    w.tno = N % 128 == 0 ? 2 : 1;
    w.tko = C % 128 == 0 ? 2 : 1;
    w.tiles = (N / (64 * w.tno)) * (K / (64 * w.tko));
    const int chunks = (M + kWM - 1) / kWM;
    const int ns = fill_rounds(w.tiles, 512, std::max(1, chunks / 4));
    w.rows = ((chunks + ns - 1) / ns) * kWM;
  }
  w.nsplit = (M + w.rows - 1) / w.rows;
  w.groups = slab_groups(w.nsplit, static_cast<int64_t>(N) * K);
  return w;
}
}  // namespace

namespace {
// The patch kernel's shapes: 3x3 / pad 1, stride 1 on 56- or 28-wide maps, stride 2 on a 56-wide map
// (the ResNet-50 64- and 128-channel stages), channels up to 128.
constexpr int kPatchMaxC = 128;

bool patch_ok(const ConvGeo& g, int M, int N, bool pro) {
  if (pro || g.ks != 3 || !(g.ksw == 0 || g.ksw == 3) || g.pad != 1 || g.C % 64 != 0 || N % 64 != 0 ||
      g.C > kPatchMaxC || M % kPP != 0 || g.RH != 0)
    return false;
  if (g.stride == 1)  // 56- / 28-wide maps
    return g.H == g.OH && g.W == g.OW && (g.W == 56 || g.W == 28) && g.OH % (kPP / g.W) == 0;
  // stride 2: the 56-wide map -> 28 x 28
  return g.stride == 2 && g.W == 56 && g.H % 2 == 0 && g.OH == g.H / 2 && g.OW == 28 && g.OH % 4 == 0;
}

struct PPlan {
  int tiles, nsplit, spp, groups;
};

PPlan pplan(const ConvGeo& g, int M, int N) {
  PPlan w{};
  w.tiles = (N / 64) * (g.C / 64);
  const int stages = M / kPP;
  const int ns = fill_rounds(w.tiles, 256, std::max(1, stages / 4));  // one 12-wave block per CU
  w.spp = (stages + ns - 1) / ns;
  w.nsplit = (stages + w.spp - 1) / w.spp;
  w.groups = slab_groups(w.nsplit, static_cast<int64_t>(N) * 9 * g.C);
  return w;
}

void slab_reduce(const ConvWgradArgs& a, int nsplit, int groups, hipStream_t s) {
  const int64_t E = static_cast<int64_t>(a.N) * a.K;
  const unsigned eb = static_cast<unsigned>((E + 255) / 256);
  void* dw = a.dw;
  if (groups) {
    float* mid = a.ws + static_cast<int64_t>(nsplit) * E;
    void* midv = mid;
    hipLaunchKernelGGL(slab_reduce_kernel<false>, dim3(eb, groups), dim3(256), 0, s, a.ws, nsplit, 16, E, midv);
    hipLaunchKernelGGL(slab_reduce_kernel<true>, dim3(eb), dim3(256), 0, s, mid, groups, groups, E, dw);
  } else {
    hipLaunchKernelGGL(slab_reduce_kernel<true>, dim3(eb), dim3(256), 0, s, a.ws, nsplit, nsplit, E, dw);
  }
}
}  // namespace

int64_t conv_wgrad_ws_geo(int M, int N, int K, const ConvGeo& g, bool pro) {
  if (patch_ok(g, M, N, pro)) {
    const PPlan w = pplan(g, M, N);
    return static_cast<int64_t>(w.nsplit + w.groups) * N * K;
  }
  return conv_wgrad_ws(M, N, K, g.C, pro);
}

int conv_wgrad_splits(int M, int N, int K, int C, bool pro) { return wplan(M, N, K, C, pro).nsplit; }
bool conv_wgrad_is_wide(int M, int N, int K, int C, bool pro) { return wplan(M, N, K, C, pro).wide != 0; }

int64_t conv_wgrad_ws(int M, int N, int K, int C, bool pro) {
  const WPlan w = wplan(M, N, K, C, pro);
  return static_cast<int64_t>(w.nsplit + w.groups) * N * K;
}

void launch_conv_wgrad(const ConvWgradArgs& a0, hipStream_t s) {
  if (a0.M <= 0) return;
  ConvWgradArgs a = a0;
  a.fd_ohw = make_fastdiv(static_cast<uint32_t>(a.g.OH * a.g.OW));
  a.fd_ow = make_fastdiv(static_cast<uint32_t>(a.g.OW));
  if (a.db == nullptr && patch_ok(a.g, a.M, a.N, a.pro != nullptr)) {
    const PPlan w = pplan(a.g, a.M, a.N);
    const int nblk = w.tiles * w.nsplit;
    if (a.g.stride == 2) hipLaunchKernelGGL((conv_wgrad_patch_kernel<56, 2>), dim3(nblk), dim3(768), 0, s, a, w.spp);
    else if (a.g.W == 56) hipLaunchKernelGGL((conv_wgrad_patch_kernel<56, 1>), dim3(nblk), dim3(768), 0, s, a, w.spp);
    else hipLaunchKernelGGL((conv_wgrad_patch_kernel<28, 1>), dim3(nblk), dim3(768), 0, s, a, w.spp);
    slab_reduce(a, w.nsplit, w.groups, s);
    return;
  }
  const WPlan w = wplan(a.M, a.N, a.K, a.g.C, a.pro != nullptr);
  const int nblk = w.tiles * w.nsplit;
  // LIN: 1x1 stride-1 pad-0 geometry (X row m = pixel m), DMA sources without the pixel decode
  const bool lin = a.g.ks == 1 && a.g.stride == 1 && a.g.pad == 0;
  const bool prol = a.g.ks == 1;  // the LDS pass maps k to the channel directly
#define PSAMD_CWW3(TN, TK, WN, WK, L)                                                                             \
  if (a.pro && prol && (WK * 32 * TK == 128 || WK * 32 * TK == 256))                                            \
    hipLaunchKernelGGL((conv_wgrad_wide_kernel<TN, TK, WN, WK, true, false, L, (WK * 32 * TK == 128 ||          \
                                                                             WK * 32 * TK == 256)>),            \
                       dim3(nblk), dim3(512), 0, s, a, w.rows);                                                  \
  else if (a.pro) hipLaunchKernelGGL((conv_wgrad_wide_kernel<TN, TK, WN, WK, true, false, L>), dim3(nblk),      \
                                     dim3(512), 0, s, a, w.rows);                                               \
  else if (a.db) hipLaunchKernelGGL((conv_wgrad_wide_kernel<TN, TK, WN, WK, false, true, L>), dim3(nblk),        \
                                    dim3(512), 0, s, a, w.rows);                                                \
  else hipLaunchKernelGGL((conv_wgrad_wide_kernel<TN, TK, WN, WK, false, false, L>), dim3(nblk), dim3(512), 0, s, \
                          a, w.rows)
#define PSAMD_CWW(TN, TK, WN, WK) \
  if (lin) { PSAMD_CWW3(TN, TK, WN, WK, true); } else { PSAMD_CWW3(TN, TK, WN, WK, false); }
#define PSAMD_CW(TN, TK, PRO, GL) \
  hipLaunchKernelGGL((conv_wgrad_kernel<TN, TK, PRO, GL>), dim3(nblk), dim3(256), 0, s, a, w.rows)
  // without the prologue both operands are plain row slices: LDS-DMA staging
#define PSAMD_CWP(TN, TK) \
  if (a.pro) { PSAMD_CW(TN, TK, true, false); } else { PSAMD_CW(TN, TK, false, true); }
  if (w.wide == 1) {
    PSAMD_CWW(2, 4, 4, 2);
  } else if (w.wide == 2) {
    PSAMD_CWW(2, 2, 4, 2);
  } else if (w.wide == 3) {
    PSAMD_CWW(2, 2, 2, 4);
  } else if (w.wide == 4) {
    PSAMD_CWW(2, 3, 2, 4);
  } else if (w.tno == 2) {
    if (w.tko == 2) { PSAMD_CWP(2, 2) } else { PSAMD_CWP(2, 1) }
  } else {
    if (w.tko == 2) { PSAMD_CWP(1, 2) } else { PSAMD_CWP(1, 1) }
  }
#undef PSAMD_CWW
#undef PSAMD_CWW3
#undef PSAMD_CWP
#undef PSAMD_CW
  if (w.wide && a.db != nullptr && a.pro == nullptr)  // bias gradient: fold the per-split column sums
    hipLaunchKernelGGL(slab_reduce_kernel<false>, dim3((a.N + 255) / 256), dim3(256), 0, s, a.dbws, w.nsplit,
                       w.nsplit, static_cast<int64_t>(a.N), static_cast<void*>(a.db));
  slab_reduce(a, w.nsplit, w.groups, s);
}

}  // namespace psamd
