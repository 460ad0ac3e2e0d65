// crc32c_lanespan.h -- records of 1..1023 B (WAL / MANIFEST physical records: type || fragment,
// db/log_writer.cc:111-121) with one lane per record and the bytes STAGED THROUGH LDS.
//
// Why: the lane-per-record kernels (crc_lanerec9/17/33) load each lane's own record window with
// 16-B loads, so every load instruction touches 64 different cache lines and the texture-address
// unit (TA) spends ~74 cycles on it against ~30 for a coalesced 1-KiB load: TA-bound at 42-51 % of
// HBM.  But a wave's 64 consecutive records of a log image are ONE contiguous span
// (records + 6-byte headers): here it is loaded with coalesced 16-B-per-lane loads (each load
// instruction 1 KiB contiguous), written to the wave's LDS region, and every lane then reads its
// own record from LDS.
//
// LDS image (160 KiB, one 256-thread workgroup = 4 waves per CU):
//   [0, 64 KiB)      T0..T3 replicated 16x: entry b of table k, replica r at b<<8 | k<<6 | r<<2 (lane
//                    l uses replica l & 15: 2-way bank conflicts, the price of fitting the staging)
//   [64, 80 KiB)     4 shift operators (16, 64, 256, 1024 B), single copy: the chain fold and the
//                    whole-wave slow path (32 = 16 twice, 128 = 64 twice, 512 = 256 twice)
//   [80, 160 KiB)    4 x 20 KiB: one staging region per wave
// A wave handles batches of 64 consecutive records (lane u: record 64b + u).  If the batch's span
// does not fit a region (records spread out, or large), it is cut into sub-batches of 32, 16, ...
// lanes (groups of consecutive lanes whose span fits: always possible, a record of the class is
// < 20 KiB); only the group's lanes hash while it is staged.  Items (sub-batches) are pipelined
// two deep in registers: while item k is hashed from LDS, items k+1 and k+2 are in flight.
// Per lane, the record is END-aligned on a grid of 4-byte words: word j = bytes [e - 4(NW - j), +4)
// built by one v_perm from two LDS dwords, bytes before p zeroed, U[z] injected at the word
// holding p (z zeroed bytes: the state entering the record is Value()'s 0xFFFFFFFF), hashed as two
// slice-by-4 chains (the last kTailB bytes separately, folded with one shift operator).  Records
// outside the class (0 B, > MAXN) are hashed by the whole wave when their batch is opened (slow
// path: global loads, the same operators; rare, so their loads may wait behind the items in flight).
#pragma once
#include "crc32c_device.h"

namespace pdb {
namespace {

constexpr uint32_t kSpanTabBytes = 64u << 10;
constexpr uint32_t kSpanOpBase = kSpanTabBytes;                   // ops: 0 = 16, 1 = 64, 2 = 256, 3 = 1024
constexpr uint32_t kSpanStageBase = kSpanOpBase + 4u * 4096u;     // 80 KiB
constexpr uint32_t kSpanWaves = 8;
constexpr uint32_t kSpanJ = 10;                                   // 1-KiB load instructions per item
constexpr uint32_t kSpanRegion = kSpanJ * 1024u;                  // staging bytes per wave
constexpr uint32_t kSpanUsable = kSpanRegion - 16u;               // span limit: reads stay inside
static_assert(kSpanStageBase + kSpanWaves * kSpanRegion == PDB_LDS_BYTES, "the whole 160 KiB");

struct LaneTabs16 {
  uint32_t t3, t2, t1, t0;  // v_perm byte 0 of the lookup address: k<<6 | replica<<2
};

__device__ __forceinline__ LaneTabs16 lane_tabs16(uint32_t lane) {
  const uint32_t r = (lane & 15u) << 2;
  return LaneTabs16{(3u << 6) | r, (2u << 6) | r, (1u << 6) | r, r};
}

// x' = shift(x, 4) ^ wnext with the 16-replica layout (the data byte lands in address bits 8..15:
// one v_perm per lookup, as step4x)
__device__ __forceinline__ uint32_t step4x16(const char* lds, const LaneTabs16& lt, uint32_t x, uint32_t wnext) {
  const uint32_t a3 = __builtin_amdgcn_perm(lt.t3, x, sel_byte(0));
  const uint32_t a2 = __builtin_amdgcn_perm(lt.t2, x, sel_byte(1));
  const uint32_t a1 = __builtin_amdgcn_perm(lt.t1, x, sel_byte(2));
  const uint32_t a0 = __builtin_amdgcn_perm(lt.t0, x, sel_byte(3));
  return xor3(xor3(lds_u32(lds, a3), lds_u32(lds, a2), lds_u32(lds, a1)), lds_u32(lds, a0), wnext);
}

__device__ __forceinline__ uint32_t span_op_x(const char* lds, uint32_t slot, uint32_t c, uint32_t y) {
  const uint32_t base = kSpanOpBase + slot * 4096u;
  const uint32_t v0 = lds_u32(lds, base + ((c & 0xffu) << 2));
  const uint32_t v1 = lds_u32(lds, base + 1024u + (((c >> 8) & 0xffu) << 2));
  const uint32_t v2 = lds_u32(lds, base + 2048u + (((c >> 16) & 0xffu) << 2));
  const uint32_t v3 = lds_u32(lds, base + 3072u + ((c >> 24) << 2));
  return xor3(xor3(v0, v1, v2), v3, y);
}

// shift(c, 16 << k) ^ y for k = 0..6 from the four slots (odd k: the slot below, twice)
__device__ __forceinline__ uint32_t span_shift_x(const char* lds, uint32_t k, uint32_t c, uint32_t y) {
  const uint32_t slot = k >> 1;
  if (k & 1u) c = span_op_x(lds, slot, c, 0u);
  return span_op_x(lds, slot, c, y);
}

__device__ __forceinline__ void stage_tables_span(char* lds, const uint32_t* __restrict__ tabs) {
  // T0..T3 x 16 replicas: 4 x 256 entries x 4 quads of 16 B
  for (uint32_t i0 = 0; i0 < 4096u; i0 += 4u * blockDim.x) {
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = i0 + threadIdx.x + j * blockDim.x;
      v[j] = i < 4096u ? tabs[(i >> 2)] : 0u;  // tabs: T0[256] T1[256] T2[256] T3[256]; i >> 2 = k*256 + b
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = i0 + threadIdx.x + j * blockDim.x;
      const uint32_t k = i >> 10, b = (i >> 2) & 255u, q = i & 3u;
      if (i < 4096u) *reinterpret_cast<u32x4*>(lds + ((b << 8) | (k << 6) | (q << 4))) = u32x4{v[j], v[j], v[j], v[j]};
    }
  }
  // operators: catalog entries 0 (16), 2 (64), 4 (256), 6 (1024)
  const u32x4* cat = reinterpret_cast<const u32x4*>(tabs + 1024);
  for (uint32_t i = threadIdx.x; i < 4u * 256u; i += blockDim.x)
    *reinterpret_cast<u32x4*>(lds + kSpanOpBase + i * 16u) = cat[(2u * (i >> 8)) * 256u + (i & 255u)];
}

// Whole-wave hash of one record of any length from global memory (Value() seed): the slow path of
// crc_sized_kernel (slow_finish) on this kernel's operator layout.  Rows of 1 KiB: lane u hashes the
// 16-B pieces at 16u + 1024k of the record front-padded with zeros to whole KiB (masked below p, U[z]
// on the piece holding p), Horner-folded with shift 1024; then a 6-level tree (16 .. 512).
__device__ __forceinline__ uint32_t span_chain16(const char* lds, const LaneTabs16& lt, uint32_t start, const uint32_t (&w)[4]) {
  uint32_t x = start ^ w[0];
  x = step4x16(lds, lt, x, w[1]);
  x = step4x16(lds, lt, x, w[2]);
  x = step4x16(lds, lt, x, w[3]);
  return step4x16(lds, lt, x, 0u);
}

__device__ __forceinline__ uint32_t span_slow_record(const char* lds, const LaneTabs16& lt, uint32_t u, uint32_t ureg,
                                                     uintptr_t p, uint32_t n) {
  if (n == 0) return 0xFFFFFFFFu;
  const uint64_t nrows = (static_cast<uint64_t>(n) + 1023u) >> 10;
  const uintptr_t vbs = p + n - (nrows << 10);  // padded start (<= p)
  const uintptr_t l4 = p & ~static_cast<uintptr_t>(3);
  uint32_t acc = 0;
  for (uint64_t r = 0; r < nrows; ++r) {
    const uintptr_t A = vbs + (r << 10) + 16u * u;  // this lane's 16 bytes
    const uint32_t s = static_cast<uint32_t>(A & 3u);
    uint32_t e[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      uintptr_t ad = A - s + 4u * (i < 4 ? static_cast<uint32_t>(i) : (s ? 4u : 3u));
      ad = ad < l4 ? l4 : ad;  // never an aligned dword wholly below p
      e[i] = gload32(ad);
    }
    const intptr_t zl0 = static_cast<intptr_t>(p - A);
    const int32_t zl = zl0 < -1 ? -1 : (zl0 > 16 ? 16 : static_cast<int32_t>(zl0));
    const uint32_t z = zl < 0 ? 0u : static_cast<uint32_t>(zl);
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t v = __builtin_amdgcn_alignbyte(e[i + 1], e[i], s);
      const uint32_t sh = z > 4u * i ? min(z - 4u * i, 4u) : 0u;
      w[i] = sh >= 4u ? 0u : (v & (0xFFFFFFFFu << (8u * sh)));
    }
    const uint32_t uz = __shfl(ureg, static_cast<uint32_t>(zl) & 15u, 64);
    const uint32_t start = (zl >= 0 && zl < 16) ? uz : 0u;
    acc = span_op_x(lds, 3, acc, span_chain16(lds, lt, start, w));  // acc = shift1024(acc) ^ row
  }
  // tree over 64 lanes, 16 B apart: shift 16 << k between partners at distance 2^k
  uint32_t y;
  y = __builtin_amdgcn_update_dpp(0u, acc, 0x101, 0xF, 0xF, false);  // row_shl:1
  if ((u & 1u) == 0) acc = span_shift_x(lds, 0, acc, y);
  y = __builtin_amdgcn_update_dpp(0u, acc, 0x102, 0xF, 0xF, false);
  if ((u & 3u) == 0) acc = span_shift_x(lds, 1, acc, y);
  y = __builtin_amdgcn_update_dpp(0u, acc, 0x104, 0xF, 0xF, false);
  if ((u & 7u) == 0) acc = span_shift_x(lds, 2, acc, y);
  y = __builtin_amdgcn_update_dpp(0u, acc, 0x108, 0xF, 0xF, false);
  if ((u & 15u) == 0) acc = span_shift_x(lds, 3, acc, y);
  y = __builtin_amdgcn_ds_swizzle(acc, 0x401F);  // lane ^ 16
  if ((u & 31u) == 0) acc = span_shift_x(lds, 4, acc, y);
  y = __builtin_amdgcn_readlane(acc, 32);
  if (u == 0) acc = span_shift_x(lds, 5, acc, y);
  return __builtin_amdgcn_readfirstlane(acc);
}

// ---- items ---------------------------------------------------------------------------------------
// A batch is 64 consecutive records (lane r of the batch registers: record 64 * batch + r).  Its
// in-class records are hashed by items: runs of up to G = floor(64 / k) consecutive records, each
// record on k consecutive lanes (lane u: record slot u / k, part c = u % k).  Per record 2k chains:
// chain i covers the words [nw - L(i + 1), nw - L i) counted from the record's END (L = kSpanL
// words), the last chain (i = 2k - 1, the head) everything before as well; part c runs chains 2c
// (A) and 2c + 1 (B).  All chains of an item run in lock step for `iters` = max(L, nw - (2k-1) L)
// steps: the head chain alone for the first iters - L, then every chain for L.  Folds: per lane
// P = shift(B, 4L) ^ A, then across the k lanes of a record shift(P[c + m], 8Lm) ^ P[c] for m = 1,
// 2, 4.  k per batch minimises steps per record for its longest in-class record (span_pick).
constexpr uint32_t kNoRec = 0x3FFFFFFFu;
constexpr uint32_t kSpanL = 16;  // words per tail chain: 64 B, the slot-1 fold

struct LaneSpanGeom {
  uint32_t k;      // lanes per record
  uint32_t g;      // records per item: floor(64 / k)
  uint32_t magic;  // ceil(65536 / k): u / k = (u * magic) >> 16 for u < 64
  uint32_t iters;  // chain steps per item
};

// max over the wave of a 32-bit value; every lane must be active
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0xB1, 0xF, 0xF, false)));
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x4E, 0xF, 0xF, false)));
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x141, 0xF, 0xF, false)));
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x140, 0xF, 0xF, false)));
  const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
  const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  return max(max(a, b), max(c, d));
}

// k for a batch whose longest in-class record has nw words: fewest steps per record, counting the
// records an item can hold (G, and what fits a staging region at ~4 nw + 8 bytes a record)
template <uint32_t KMAX>
__device__ __forceinline__ LaneSpanGeom span_pick(uint32_t nw) {
  const float fit = static_cast<float>(kSpanUsable) * __builtin_amdgcn_rcpf(static_cast<float>(4u * nw + 8u));
  uint32_t gfit = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(fit)));
  gfit = gfit ? gfit : 1u;
  LaneSpanGeom best{1u, 64u, 65536u, kSpanL};
  uint32_t best_eff = 1u;
#pragma unroll
  for (uint32_t k = 1; k <= KMAX; ++k) {
    const uint32_t g = 64u / k;
    const uint32_t geff = g < gfit ? g : gfit;
    const int32_t h = static_cast<int32_t>(nw) - static_cast<int32_t>((2u * k - 1u) * kSpanL);
    const uint32_t it = h > static_cast<int32_t>(kSpanL) ? static_cast<uint32_t>(h) : kSpanL;
    if (k == 1 || it * best_eff < best.iters * geff) {
      best = LaneSpanGeom{k, g, (65536u + k - 1u) / k, it};
      best_eff = geff;
    }
  }
  return best;
}

struct SpanItem {
  uint64_t batch;   // records 64 * batch + r
  uintptr_t lo;     // 16-B aligned global address of region byte 0
  uint32_t hi;      // local end: max over the item's records (0: nothing to hash)
  uint32_t k, iters;
  bool valid;
  uint32_t r, c;               // per lane: record slot in the batch, part
  uint32_t p_loc, e_loc, pre;  // per lane: local start (kNoRec: no record), local end, sink word
};

template <class Src, class Sink, uint32_t MAXN>
__global__ __launch_bounds__(kSpanWaves * 64) void crc_lanespan_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                                       uint64_t nblk, Sink sink) {
  static_assert(MAXN + 32u <= kSpanUsable, "a record of the class must fit a region");
  constexpr uint32_t KMAX = (MAXN + 8u * kSpanL - 1u) / (8u * kSpanL);  // 2k chains cover MAXN: 2, 4, 8
  static_assert(KMAX >= 1 && KMAX <= 8, "tree folds for up to 8 lanes per record");
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  stage_tables_span(lds, tabs);
  const uint32_t u = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ureg = tabs[PDB_UNSHIFT_OFF + (u & 15u)];
  __syncthreads();
  const LaneTabs16 lt = lane_tabs16(u);
  char* region = lds + kSpanStageBase + wv * kSpanRegion;
  const uintptr_t dummy = reinterpret_cast<uintptr_t>(tabs);  // >= 4 KiB + 256 B of valid bytes
  const uint64_t nbat = (nblk + 63u) >> 6;
  const uint64_t W = static_cast<uint64_t>(gridDim.x) * kSpanWaves;
  uint64_t bnext = static_cast<uint64_t>(blockIdx.x) * kSpanWaves + wv;  // next batch to open
  if (bnext >= nbat) return;  // wave-uniform; no barrier below

  auto idx = [&](uint64_t bb) -> uint64_t {
    const uint64_t i = (bb << 6) + u;
    return i < nblk ? i : nblk - 1;
  };
  // the next batch's descriptors and sink words, in flight; reloaded by every next_item call (the
  // same address when no batch was opened) so no load is ever consumed right after it is issued
  typename Src::Raw raw_next = src.load(idx(bnext));
  uint32_t pre_next = SinkOps<Sink>::pre(sink, idx(bnext), BlkDesc{nullptr, 0u, 0u});
  uint64_t bcur = 0;
  bool have_batch = false;
  uintptr_t bp = 0;      // per lane: record start
  uint32_t bn = 0;       // per lane: record length
  bool bfast = false;    // per lane: in the class (hashed from LDS)
  uint32_t bpre = 0;     // per lane: the sink's word
  uint64_t bfastm = 0;   // in-class records
  uint64_t bbroken = 0;  // bit r: records r and r + 1 may not share an item
  uint32_t bcursor = 64;
  LaneSpanGeom bg{1u, 64u, 65536u, kSpanL};

  // make the prefetched batch current; records outside the class are hashed here by the whole
  // wave (rare: their loads wait behind the items in flight)
  auto open_batch = [&]() -> bool {
    if (bnext >= nbat) return false;
    keep_alive(raw_next);
    const BlkDesc d = src.lane(raw_next);
    bpre = pre_next;
    bcur = bnext;
    bnext += W;
    const uint64_t i = (bcur << 6) + u;
    const bool valid = i < nblk;
    bp = reinterpret_cast<uintptr_t>(d.p);
    bn = d.n;
    bfast = valid && (d.n - 1u) <= MAXN - 1u && d.init_raw == 0xFFFFFFFFu;
    uint64_t sb = __builtin_amdgcn_ballot_w64(valid && !bfast);
    const uint32_t plo = static_cast<uint32_t>(bp), phi = static_cast<uint32_t>(static_cast<uint64_t>(bp) >> 32);
    while (sb) {
      const uint32_t k = static_cast<uint32_t>(__builtin_ctzll(sb));
      sb &= sb - 1;
      const uintptr_t sp = static_cast<uintptr_t>(uniform64(__builtin_amdgcn_readlane(plo, k), __builtin_amdgcn_readlane(phi, k)));
      const uint32_t sn = __builtin_amdgcn_readlane(bn, k);
      const uint32_t rs = span_slow_record(lds, lt, u, ureg, sp, sn);
      if (u == 0)
        SinkOps<Sink>::put(sink, (bcur << 6) + k, rs, BlkDesc{reinterpret_cast<const uint8_t*>(sp), sn, 0xFFFFFFFFu},
                           __builtin_amdgcn_readlane(bpre, k));
    }
    bfastm = __builtin_amdgcn_ballot_w64(bfast);
    // link r -> r + 1: both in the class, ascending, at most 64 B apart -- every 16-B chunk an item
    // stages lies within 64 B of a record byte (a log image: 6-byte headers, <= 6-byte trailers)
    const uint32_t np_lo = __shfl_down(plo, 1, 64), np_hi = __shfl_down(phi, 1, 64);
    const uintptr_t pn = static_cast<uintptr_t>((static_cast<uint64_t>(np_hi) << 32) | np_lo);
    const uint32_t fn = __shfl_down(bfast ? 1u : 0u, 1, 64);
    const bool link_ok = bfast && fn && pn >= bp && pn <= bp + bn + 64u;
    bbroken = __builtin_amdgcn_ballot_w64(!link_ok && u < 63u);
    const uint32_t nw = wave_max_u32(bfast ? (bn + 3u) >> 2 : 0u);
    bg = span_pick<KMAX>(nw ? nw : 1u);
    bcursor = 0;
    return true;
  };

  // the next item: the next run of in-class records of the current batch (or of the next batch);
  // every field is set on every path (a partially written item ends up in scratch)
  auto next_item = [&](bool want) -> SpanItem {
    SpanItem it;
    it.valid = false;
    it.batch = bcur;
    it.lo = dummy;
    it.hi = 0;
    it.k = bg.k;
    it.iters = bg.iters;
    it.r = u;
    it.c = 0;
    it.p_loc = kNoRec;
    it.e_loc = 0;
    it.pre = 0;
    if (!want) return it;
    uint64_t rem = (have_batch && bcursor < 64u) ? (bfastm & (~0ull << bcursor)) : 0ull;
    if (rem == 0) {
      if (!open_batch()) return it;
      have_batch = true;
      rem = bfastm;
    }
    raw_next = src.load(idx(bnext < nbat ? bnext : bcur));
    pre_next = SinkOps<Sink>::pre(sink, idx(bnext < nbat ? bnext : bcur), BlkDesc{nullptr, 0u, 0u});
    it.valid = true;
    it.batch = bcur;
    it.k = bg.k;
    it.iters = bg.iters;
    if (rem == 0) {  // every record of the batch was outside the class: an empty item
      bcursor = 64;
      return it;
    }
    const uint32_t g0 = static_cast<uint32_t>(__builtin_ctzll(rem));
    const uint64_t br = bbroken >> g0;
    const uint32_t m1 = br ? static_cast<uint32_t>(__builtin_ctzll(br)) + 1u : 64u - g0;
    const uint32_t plo = static_cast<uint32_t>(bp), phi = static_cast<uint32_t>(static_cast<uint64_t>(bp) >> 32);
    const uintptr_t lo = static_cast<uintptr_t>(uniform64(__builtin_amdgcn_readlane(plo, g0), __builtin_amdgcn_readlane(phi, g0))) &
                         ~static_cast<uintptr_t>(15);
    const uint64_t over = __builtin_amdgcn_ballot_w64(bfast && u >= g0 && (bp + bn - lo) > kSpanUsable) >> g0;
    const uint32_t m2 = over ? static_cast<uint32_t>(__builtin_ctzll(over)) : 64u;
    const uint32_t m = min(min(bg.g, m1), m2);
    bcursor = g0 + m;
    const uint32_t slot = (u * bg.magic) >> 16;
    const uint32_t c = u - slot * bg.k;
    const bool act = slot < m;
    const uint32_t rl = act ? g0 + slot : u;
    const uintptr_t pr = static_cast<uintptr_t>((static_cast<uint64_t>(__shfl(phi, rl, 64)) << 32) | __shfl(plo, rl, 64));
    const uint32_t nr = __shfl(bn, rl, 64);
    it.pre = __shfl(bpre, rl, 64);
    it.r = rl;
    it.c = c;
    it.lo = lo;
    it.p_loc = act ? static_cast<uint32_t>(pr - lo) : kNoRec;
    it.e_loc = act ? static_cast<uint32_t>(pr + nr - lo) : 0u;
    it.hi = wave_max_u32(it.e_loc);
    return it;
  };

  // loads of one item: kSpanJ unconditional 16-B loads (1 KiB contiguous per instruction); chunks
  // wholly past the item's last byte read the dummy line instead
  auto issue = [&](u32x4 (&A)[kSpanJ], const SpanItem& it) {
    const uint32_t hi = it.hi;  // 0 for an invalid or empty item
    const uintptr_t lo = it.lo;
#pragma unroll
    for (uint32_t j = 0; j < kSpanJ; ++j) {
      const uint32_t off = 1024u * j + 16u * u;
      A[j] = gload128<true>(off < hi ? lo + off : dummy);
    }
  };
  // every chunk is written, the dummy ones too: a load whose register is never read stays
  // outstanding, and the compiler then drains the counter before the register is reloaded
  auto to_lds = [&](const u32x4 (&A)[kSpanJ]) {
#pragma unroll
    for (uint32_t j = 0; j < kSpanJ; ++j) *reinterpret_cast<u32x4*>(region + 1024u * j + 16u * u) = A[j];
  };
  // hash an item staged in the region
  auto hash = [&](const SpanItem& it) {
    if (it.hi == 0) return;
    const uint32_t k = it.k, iters = it.iters, lim = iters - kSpanL;
    const int32_t e = static_cast<int32_t>(it.e_loc);
    const int32_t pl = static_cast<int32_t>(it.p_loc);
    const bool head = it.c == k - 1u;
    const uint32_t sel = static_cast<uint32_t>(e & 3) * 0x01010101u + 0x03020100u;
    const uint32_t uz = __shfl(ureg, static_cast<uint32_t>(pl - e) & 3u, 64);
    // word at byte s (s = e mod 4): bytes of the dword pair (D[s >> 2], D[(s >> 2) + 1]), masked
    // below p; the word holding p injects U[z] (z bytes of it before p)
    auto dword = [&](int32_t q) -> uint32_t { return lds_u32(region, static_cast<uint32_t>(q < 0 ? 0 : q) << 2); };
    auto word = [&](int32_t s, uint32_t& lo_dw) -> uint32_t {
      const uint32_t hi_dw = dword((s >> 2) + 1);
      const uint32_t w = __builtin_amdgcn_perm(hi_dw, lo_dw, sel);
      lo_dw = hi_dw;
      const int32_t z = pl - s;
      const uint32_t zc = static_cast<uint32_t>(z < 0 ? 0 : (z > 4 ? 4 : z));
      const uint32_t m = static_cast<uint32_t>(0xFFFFFFFFull << (8u * zc));
      return (w & m) ^ (static_cast<uint32_t>(z) < 4u ? uz : 0u);
    };
    const int32_t sA0 = e - static_cast<int32_t>(8u * kSpanL * it.c) - 4 * static_cast<int32_t>(iters);
    const int32_t sB0 = sA0 - 4 * static_cast<int32_t>(kSpanL);
    uint32_t lb = dword(sB0 >> 2);
    uint32_t xb = word(sB0, lb);
    if (lim > 0) {  // the head chain's first words (junk on the other lanes, dropped)
      for (uint32_t t = 1; t < lim; ++t) xb = step4x16(lds, lt, xb, word(sB0 + 4 * static_cast<int32_t>(t), lb));
      xb = head ? xb : 0u;
      xb = step4x16(lds, lt, xb, word(sB0 + 4 * static_cast<int32_t>(lim), lb));
    }
    const int32_t sa = sA0 + 4 * static_cast<int32_t>(lim);
    const int32_t sb = sB0 + 4 * static_cast<int32_t>(lim);
    uint32_t la = dword(sa >> 2);
    uint32_t xa = word(sa, la);
#pragma unroll
    for (uint32_t t = 1; t < kSpanL; ++t) {
      xa = step4x16(lds, lt, xa, word(sa + 4 * static_cast<int32_t>(t), la));
      xb = step4x16(lds, lt, xb, word(sb + 4 * static_cast<int32_t>(t), lb));
    }
    const uint32_t ca = step4x16(lds, lt, xa, 0u), cb = step4x16(lds, lt, xb, 0u);
    uint32_t P = span_op_x(lds, 1, cb, ca);  // shift(B, 64 B) ^ A
#pragma unroll
    for (uint32_t lvl = 0; lvl < 3; ++lvl) {
      const uint32_t m = 1u << lvl;
      if (m >= k) break;
      const uint32_t y = __shfl_down(P, m, 64);  // part c + m: the 128 m bytes before
      if ((it.c & (2u * m - 1u)) == 0 && it.c + m < k) P = span_shift_x(lds, 3u + lvl, y, P);
    }
    if (it.c == 0 && it.p_loc != kNoRec)
      SinkOps<Sink>::put(sink, (it.batch << 6) + it.r, P, BlkDesc{nullptr, 0u, 0xFFFFFFFFu}, it.pre);
  };

  // ---- pipeline: the next item's loads in flight while one is hashed ------------------------------
  // (one register array: with two, the compiler's wait counting across the loop's back edge drains
  // both arrays at the loop head; eight waves per CU keep ~70 KiB in flight per CU)
  u32x4 A[kSpanJ];
  SpanItem cur = next_item(true);
  issue(A, cur);
  while (cur.valid) {
    to_lds(A);
    const SpanItem nxt = next_item(true);
    issue(A, nxt);
    hash(cur);
    cur = nxt;
  }
}

// grid: one wave per batch of 64 records, 8 waves per workgroup, at most one workgroup per CU
inline uint32_t grid_span(const LaunchGeom& g, uint64_t nblk) {
  const uint64_t want = ((nblk + 63) / 64 + kSpanWaves - 1) / kSpanWaves;
  return static_cast<uint32_t>(want < g.grid ? (want ? want : 1) : g.grid);
}

// Records of 1..1023 B by class (the class bounds the lanes per record: 2, 4, 8); longer ones, and
// empty ones, take the whole-wave path.
template <class Src, class Sink>
void launch_lanespan(const LaunchGeom& g, const uint32_t* d_tables, const Src& src, uint64_t nblk, uint32_t cls,
                     const Sink& sink, hipStream_t s) {
  const dim3 grid(grid_span(g, nblk)), block(kSpanWaves * 64);
  if (cls <= 256u)
    hipLaunchKernelGGL((crc_lanespan_kernel<Src, Sink, 256>), grid, block, 0, s, d_tables, src, nblk, sink);
  else if (cls <= 512u)
    hipLaunchKernelGGL((crc_lanespan_kernel<Src, Sink, 512>), grid, block, 0, s, d_tables, src, nblk, sink);
  else
    hipLaunchKernelGGL((crc_lanespan_kernel<Src, Sink, 1023>), grid, block, 0, s, d_tables, src, nblk, sink);
}

}  // namespace
}  // namespace pdb
