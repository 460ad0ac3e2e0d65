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
constexpr uint32_t kSpanWaves = 4;
constexpr uint32_t kSpanJ = 20;                                   // 1-KiB load instructions per item
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

// One item: a group of consecutive lanes of a batch whose records' bytes [lo, lo + 1 KiB x chunks)
// are loaded into the wave's LDS region.  Per lane: the record's local start / end in the region
// (p_loc = kNoRec for lanes outside the group or outside the class) and the sink's preloaded word.
constexpr uint32_t kNoRec = 0x3FFFFFFFu;

struct SpanItem {
  uint64_t batch;   // records 64*batch + lane
  uintptr_t lo;     // 16-B aligned global address of region byte 0
  uint32_t nw;      // words to hash: max over the group's records of ceil(n / 4)
  bool valid;
  uint32_t p_loc, e_loc, pre;  // per lane
};

// Lanes per item for a batch: the largest power of two B such that every group of B consecutive
// lanes (a) spans at most kSpanUsable bytes from its first record's 16-B line, and (b) holds
// records in ascending address order with gaps of at most 64 B between neighbours -- so every
// 16-B chunk loaded lies within 64 B of a record byte, on a page that holds one: the staging
// never reads memory a caller's blocks do not touch (a log image: 6-byte headers, <= 6-byte block
// trailers between records).  A lane outside the class breaks the chain (groups split around it).
template <uint32_t kUsable>
__device__ __forceinline__ uint32_t span_group_size(uint32_t u, bool fast, uintptr_t p, uint32_t n) {
  const uintptr_t e = p + n;
  // link u -> u+1
  const uint32_t np_lo = __shfl_down(static_cast<uint32_t>(p), 1, 64);
  const uint32_t np_hi = __shfl_down(static_cast<uint32_t>(static_cast<uint64_t>(p) >> 32), 1, 64);
  const uintptr_t pn = static_cast<uintptr_t>((static_cast<uint64_t>(np_hi) << 32) | np_lo);
  const uint32_t fn = __shfl_down(fast ? 1u : 0u, 1, 64);
  const bool link_ok = fast && fn && pn >= p && pn <= e + 64u;
  const uint64_t broken = __builtin_amdgcn_ballot_w64(!link_ok && u < 63u);
  uintptr_t mn = fast ? p : ~static_cast<uintptr_t>(0);
  uintptr_t mx = fast ? e : 0;
  uint32_t best = 1;
#pragma unroll
  for (uint32_t m = 1; m < 64; m <<= 1) {
    const uint64_t omn = static_cast<uint64_t>(__shfl_xor(static_cast<uint32_t>(mn), m, 64)) |
                         (static_cast<uint64_t>(__shfl_xor(static_cast<uint32_t>(static_cast<uint64_t>(mn) >> 32), m, 64)) << 32);
    const uint64_t omx = static_cast<uint64_t>(__shfl_xor(static_cast<uint32_t>(mx), m, 64)) |
                         (static_cast<uint64_t>(__shfl_xor(static_cast<uint32_t>(static_cast<uint64_t>(mx) >> 32), m, 64)) << 32);
    mn = omn < mn ? static_cast<uintptr_t>(omn) : mn;
    mx = omx > mx ? static_cast<uintptr_t>(omx) : mx;
    const uint32_t B = m << 1;  // group size after this level
    const bool span_ok = mx == 0 || (mx - (mn & ~static_cast<uintptr_t>(15))) <= kUsable;
    uint64_t inner = ~0ull;  // link positions inside a group of B lanes (not the last lane of a group)
#pragma unroll
    for (uint32_t g = B - 1; g < 64; g += B) inner &= ~(1ull << g);
    if (__builtin_amdgcn_ballot_w64(!span_ok) == 0 && (broken & inner) == 0) best = B;
    else break;
  }
  return best;
}

template <class Src, class Sink, uint32_t MAXN, uint32_t kTailB>
__global__ __launch_bounds__(kSpanWaves * 64) void crc_lanespan_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                                       uint64_t nblk, Sink sink) {
  static_assert(MAXN + 64u <= kSpanUsable, "a record of the class must fit a region");
  static_assert(kTailB == 64u || kTailB == 256u, "the tail chain folds with slot 1 (64) or 2 (256)");
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
  constexpr uint32_t kTailW = kTailB / 4u;
  constexpr uint32_t kTailSlot = kTailB == 64u ? 1u : 2u;

  auto idx = [&](uint64_t bb) -> uint64_t {
    const uint64_t i = (bb << 6) + u;
    return i < nblk ? i : nblk - 1;
  };
  // ---- the batch whose items are being issued --------------------------------------------------
  typename Src::Raw raw_next = src.load(idx(bnext));
  uint64_t bcur = 0;
  bool have_batch = false;
  uintptr_t bp = 0;         // per lane: record start
  uint32_t bn = 0;          // per lane: record length
  bool bfast = false;       // per lane: in the class (hashed from LDS)
  uint32_t bpre = 0;        // per lane: the sink's preloaded word
  uint32_t bgroup = 64;     // lanes per item of this batch
  uint32_t bnext_item = 0;  // next group to issue

  // make the prefetched descriptors current, prefetch the next batch's; records outside the class
  // are hashed here by the whole wave (rare: their loads wait behind the items in flight)
  auto open_batch = [&]() -> bool {
    if (bnext >= nbat) return false;
    keep_alive(raw_next);
    const BlkDesc d = src.lane(raw_next);
    bcur = bnext;
    bnext += W;
    raw_next = src.load(idx(bnext < nbat ? bnext : bcur));  // unconditional
    const uint64_t i = (bcur << 6) + u;
    const bool valid = i < nblk;
    bp = reinterpret_cast<uintptr_t>(d.p);
    bn = d.n;
    bfast = valid && (d.n - 1u) <= MAXN - 1u && d.init_raw == 0xFFFFFFFFu;
    bpre = SinkOps<Sink>::pre(sink, idx(bcur), d);
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
    bgroup = __builtin_amdgcn_readfirstlane(span_group_size<kSpanUsable>(u, bfast, bp, bn));
    bnext_item = 0;
    return true;
  };

  // the next item (a group with at least one record in the class), opening batches as needed
  auto next_item = [&](SpanItem& it) -> bool {
    for (;;) {
      if (!have_batch || bnext_item * bgroup >= 64u) {
        if (!open_batch()) return false;
        have_batch = true;
      }
      const uint32_t g0 = bnext_item * bgroup;
      ++bnext_item;
      const bool mine = bfast && u >= g0 && u < g0 + bgroup;
      if (__builtin_amdgcn_ballot_w64(mine) == 0) continue;
      uintptr_t mn = mine ? bp : ~static_cast<uintptr_t>(0);
      uint32_t w = mine ? (bn + 3u) >> 2 : 0u;
#pragma unroll
      for (uint32_t m = 1; m < 64; m <<= 1) {
        const uint64_t o = static_cast<uint64_t>(__shfl_xor(static_cast<uint32_t>(mn), m, 64)) |
                           (static_cast<uint64_t>(__shfl_xor(static_cast<uint32_t>(static_cast<uint64_t>(mn) >> 32), m, 64)) << 32);
        mn = o < mn ? static_cast<uintptr_t>(o) : mn;
        const uint32_t ow = __shfl_xor(w, m, 64);
        w = ow > w ? ow : w;
      }
      it.lo = static_cast<uintptr_t>(uniform64(static_cast<uint32_t>(mn), static_cast<uint32_t>(static_cast<uint64_t>(mn) >> 32))) &
              ~static_cast<uintptr_t>(15);
      it.nw = __builtin_amdgcn_readfirstlane(w);
      it.batch = bcur;
      it.valid = true;
      it.p_loc = mine ? static_cast<uint32_t>(bp - it.lo) : kNoRec;
      it.e_loc = mine ? static_cast<uint32_t>(bp + bn - it.lo) : 0u;
      it.pre = bpre;
      return true;
    }
  };

  // loads of one item: kSpanJ unconditional 16-B loads (1 KiB contiguous per instruction); chunks
  // wholly past the group's last byte read the dummy line instead
  auto issue = [&](u32x4 (&A)[kSpanJ], const SpanItem& it, uint32_t& nchunks) {
    uint32_t hi = it.valid ? it.e_loc : 0u;  // local end, max over lanes
#pragma unroll
    for (uint32_t m = 1; m < 64; m <<= 1) {
      const uint32_t o = __shfl_xor(hi, m, 64);
      hi = o > hi ? o : hi;
    }
    hi = __builtin_amdgcn_readfirstlane(hi);
    nchunks = (hi + 1023u) >> 10;
    const uintptr_t lo = it.valid ? it.lo : dummy;
#pragma unroll
    for (uint32_t j = 0; j < kSpanJ; ++j) {
      const uint32_t off = 1024u * j + 16u * u;
      A[j] = gload128<true>(off < hi ? lo + off : dummy);
    }
  };
  auto to_lds = [&](const u32x4 (&A)[kSpanJ], uint32_t nchunks) {
#pragma unroll
    for (uint32_t j = 0; j < kSpanJ; ++j)
      if (j < nchunks) *reinterpret_cast<u32x4*>(region + 1024u * j + 16u * u) = A[j];
  };
  // hash an item staged in the region: chain A = the words before the last kTailB bytes, chain B =
  // the tail, folded as shift(A, kTailB) ^ B
  auto hash = [&](const SpanItem& it) {
    const int32_t nw = static_cast<int32_t>(it.nw);
    const int32_t e = static_cast<int32_t>(it.e_loc);
    const int32_t pl = static_cast<int32_t>(it.p_loc);
    const uint32_t sel = static_cast<uint32_t>(e & 3) * 0x01010101u + 0x03020100u;
    const uint32_t uz = __shfl(ureg, static_cast<uint32_t>(pl - e) & 3u, 64);
    // word j starts at s_j = e - 4 (nw - j): bytes sh.. of the dword pair (D[q_j], D[q_j + 1]),
    // q_j = s_j >> 2 (floor), masked below p; the word holding p injects U[z]
    auto dword = [&](int32_t q) -> uint32_t { return lds_u32(region, static_cast<uint32_t>(q < 0 ? 0 : q) << 2); };
    auto word = [&](int32_t j, uint32_t& lo_dw) -> uint32_t {
      const int32_t s = e - 4 * (nw - j);
      const uint32_t hi_dw = dword((s >> 2) + 1);
      const uint32_t w = __builtin_amdgcn_perm(hi_dw, lo_dw, sel);
      lo_dw = hi_dw;
      const int32_t z = pl - s;  // bytes of the word before the record
      const uint32_t m = z <= 0 ? 0xFFFFFFFFu : (z >= 4 ? 0u : (0xFFFFFFFFu << (8u * static_cast<uint32_t>(z))));
      return (w & m) ^ ((z >= 0 && z < 4) ? uz : 0u);
    };
    const int32_t ntail = nw < static_cast<int32_t>(kTailW) ? nw : static_cast<int32_t>(kTailW);
    const int32_t nhead = nw - ntail;
    uint32_t la = dword((e - 4 * nw) >> 2), lb = dword((e - 4 * ntail) >> 2);
    uint32_t xa = nhead > 0 ? word(0, la) : 0u;
    uint32_t xb = word(nhead, lb);
    for (int32_t k = 1; k < ntail; ++k) {
      if (k < nhead) xa = step4x16(lds, lt, xa, word(k, la));
      xb = step4x16(lds, lt, xb, word(nhead + k, lb));
    }
    for (int32_t k = ntail; k < nhead; ++k) xa = step4x16(lds, lt, xa, word(k, la));
    xb = step4x16(lds, lt, xb, 0u);
    uint32_t c = xb;
    if (nhead > 0) c = span_op_x(lds, kTailSlot, step4x16(lds, lt, xa, 0u), xb);
    if (it.p_loc != kNoRec)
      SinkOps<Sink>::put(sink, (it.batch << 6) + u, c, BlkDesc{nullptr, 0u, 0xFFFFFFFFu}, it.pre);
  };

  // ---- pipeline: two items in flight while one is hashed ---------------------------------------
  SpanItem I0{}, I1{}, I2{};
  u32x4 A[kSpanJ], B[kSpanJ];
  uint32_t na = 0, nb = 0;
  I0.valid = next_item(I0);
  issue(A, I0, na);
  I1.valid = I0.valid && next_item(I1);
  issue(B, I1, nb);
  while (I0.valid) {
    to_lds(A, na);
    I2.valid = I1.valid && next_item(I2);
    issue(A, I2, na);  // A is free again: the item after next
    hash(I0);
    if (!I1.valid) break;
    to_lds(B, nb);
    I0 = I2;
    I2.valid = I0.valid && next_item(I2);
    issue(B, I2, nb);
    hash(I1);
    I1 = I2;
  }
}

// grid: one wave per batch of 64 records, 4 waves per workgroup, at most one workgroup per CU
inline uint32_t grid_span(const LaunchGeom& g, uint64_t nblk) {
  const uint64_t want = ((nblk + 63) / 64 + kSpanWaves - 1) / kSpanWaves;
  return static_cast<uint32_t>(want < g.grid ? (want ? want : 1) : g.grid);
}

// Records of 1..1023 B by class: <= 256 B (tail chain 64 B), 257..512 and 513..1023 B (tail 256 B).
template <class Src, class Sink>
void launch_lanespan(const LaunchGeom& g, const uint32_t* d_tables, const Src& src, uint64_t nblk, uint32_t cls,
                     const Sink& sink, hipStream_t s) {
  const dim3 grid(grid_span(g, nblk)), block(kSpanWaves * 64);
  if (cls <= 256u)
    hipLaunchKernelGGL((crc_lanespan_kernel<Src, Sink, 256, 64>), grid, block, 0, s, d_tables, src, nblk, sink);
  else if (cls <= 512u)
    hipLaunchKernelGGL((crc_lanespan_kernel<Src, Sink, 512, 256>), grid, block, 0, s, d_tables, src, nblk, sink);
  else
    hipLaunchKernelGGL((crc_lanespan_kernel<Src, Sink, 1023, 256>), grid, block, 0, s, d_tables, src, nblk, sink);
}

}  // namespace
}  // namespace pdb
