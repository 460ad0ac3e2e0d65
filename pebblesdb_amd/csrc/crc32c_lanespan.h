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
// LDS image (160 KiB, one 704-thread workgroup = 11 waves per CU, for the <= 256-B class):
//   [0, 64 KiB)      256 entry blocks of 256 B, block b at b << 8 (v_perm puts a state byte in
//                    address bits 8..15 in one instruction):
//                    [0, 128)    T0..T3 x 8 replicas: T_k replica r at dword k * 8 + r, bank
//                                k * 8 + r.  In lookup instruction i, lane quarter q ((lane >> 3)
//                                & 3) reads table (q + i) & 3, replica lane & 7: the four quarters
//                                of each 32-lane group read four tables in four disjoint bank
//                                ranges, every lookup bank-conflict free on 32 KiB of tables.
//                    [128, 256)  8 shift operators (16, 32, 64, 256, 1024 and the class's three
//                                part operators), one copy, sub-table j of operator s at dword
//                                32 + (((b >> 2) ^ (4 s + j)) & 31): scrambled by b so a lookup's
//                                lanes spread over the banks, and the address is one v_perm
//                                ([b, b, 0, 0]) and one v_bitop3 ((x & 0xFF7C) ^ const) away.
//   [64, 160 KiB)    11 x 8928 B: one staging region per wave (64 records of a 100-B-value log, 138 B
//                    each with their headers, fit one)
// A wave handles batches of 64 consecutive records; their records are hashed by items (runs of
// consecutive records whose span fits a region, each record on k lanes: see "items" below).  The
// next item's loads are in flight while one is hashed.  Per lane, a record part is a run of the
// region's dwords counted from the record's last one (whose bytes past the record are masked; the
// finishing step then shifts by the record bytes it holds) and hashed as two interleaved slice-by-4
// chains (four until round 5); the dword holding the record's first byte p is masked below p and injects U[z] (z masked
// bytes: the state entering the record is Value()'s 0xFFFFFFFF), and it REPLACES the state of its
// chain, so no word before it needs masking.  Records outside the class (0 B, > MAXN)
// are hashed by the whole wave when their batch is opened (slow path: global loads, the same
// operators; rare, so their loads may wait behind the item in flight).
#pragma once
#include "crc32c_device.h"

namespace pdb {
namespace {

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr uint32_t kSpanStageBase = 64u << 10;                    // tables and operators below
// staging geometry per class: waves per CU, 1-KiB load chunks per item and the region size (11 x
// 8928 B for <= 256-B records: 64 records of a 100-B-value log, 8832 B, fit a region, whose last
// chunk is staged by its first 46 lanes only; 12 x 8 KiB for the longer classes, whose items hold
// 8..21 records on 3..8 lanes each -- more waves hide more of the hash's latency)
//
// and the part geometry (see "items" below): chains A, B, C of kLC = 8 words and chain D of kLD
// words, kPart = 3 kLC + kLD words per lane.  33-word parts (kLD = 9) for <= 256 B (a 131-B record
// on one lane) and 513..1023 B (up to 8 lanes); 27-word parts (kLD = 3) for 257..512 B, where 4
// lanes of 27 words cover a 431-B record exactly instead of 4 x 33 = 132 words for its 108.
// The 1024..1152-B class takes 11 x 8928 B too: eight 1062-B records (1055-B fragments + headers)
// do not fit 8 KiB, so 8-KiB items held 7 records on 56 of the 64 lanes (+2.5 % with 9 KiB,
// −4..−9 % for the 512 and 1023 classes, whose 8 records fit 8 KiB; profiles/r03_wide/).  11 waves
// of 8928 B instead of 10 of 9 KiB (round 5): profiles/r05/ab/ab_11waves.log.
template <uint32_t MAXN>
struct SpanStage {
  static constexpr bool k9 = MAXN <= 256u || MAXN > 1023u;
  static constexpr uint32_t kWaves = k9 ? 11u : 12u;
  static constexpr uint32_t kJ = k9 ? 9u : 8u;
  static constexpr uint32_t kRegion = k9 ? 8928u : 8192u;  // (a multiple of 16 B)
  static constexpr uint32_t kLastLanes = (kRegion - 1024u * (kJ - 1u)) / 16u;  // lanes staging the last chunk
  static_assert(kRegion % 16u == 0 && kLastLanes >= 1u && kLastLanes <= 64u, "the last chunk ends the region");
  static constexpr uint32_t kUsable = kRegion - 16u;  // span limit: reads stay inside
  static_assert((64u << 10) + kWaves * kRegion <= PDB_LDS_BYTES, "fits the 160 KiB");
  static constexpr uint32_t kLC = 8;                                // words of chains A, B, C (the 32-B folds)
  static constexpr uint32_t kLD = MAXN > 256u && MAXN <= 512u ? 3u : 9u;  // words of chain D (not the head)
  static constexpr uint32_t kPart = 3 * kLC + kLD;                  // odd: a record's k lanes on k banks
  static constexpr uint32_t kNI = kLD > kLC ? kLD : kLC;            // lock-step steps of a part
  static constexpr uint32_t kOpSet = kLD == 9u ? 0u : 3u;           // its part operators in the table source
};
// operator slots: 5..7 and 0 shift by 1, 2, 4 and 3 parts of the kernel's class (the pre-shifted
// cross-lane fold; the slow path's shift 16 is four table steps: it is rare, and the fold runs once
// per item)
constexpr uint32_t kOpP3 = 0, kOp32 = 1, kOp64 = 2, kOp256 = 3, kOp1024 = 4, kOpP1 = 5, kOpP2 = 6, kOpP4 = 7;

// shift(c, D) ^ y for the operator in slot `slot` (byte j of c indexes sub-table j)
__device__ __forceinline__ uint32_t span_op_x(const char* lds, uint32_t slot, uint32_t c, uint32_t y) {
  uint32_t v[4];
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t bb = __builtin_amdgcn_perm(0u, c, 0x0C0C0000u | (j << 8) | j);  // [b_j, b_j, 0, 0]
    v[j] = lds_u32(lds, (bb & 0xFF7Cu) ^ (128u | ((4u * slot + j) << 2)));
  }
  return xor3(xor3(v[0], v[1], v[2]), v[3], y);
}

// shift(c, 16 << k) ^ y for k = 0..5 (16, 32, 64, 64 x 2, 256, 256 x 2); shift 16 is four table
// steps (slot 0 holds the 3-part operator)
template <class TP>
__device__ __forceinline__ uint32_t span_shift_x(const char* lds, const typename TP::LT& lt, uint32_t k, uint32_t c,
                                                 uint32_t y) {
  switch (k) {
    case 0:
      return TP::step(lds, lt, TP::step(lds, lt, TP::step(lds, lt, TP::step(lds, lt, c, 0u), 0u), 0u), y);
    case 1: return span_op_x(lds, kOp32, c, y);
    case 2: return span_op_x(lds, kOp64, c, y);
    case 3: return span_op_x(lds, kOp64, span_op_x(lds, kOp64, c, 0u), y);
    case 4: return span_op_x(lds, kOp256, c, y);
    default: return span_op_x(lds, kOp256, span_op_x(lds, kOp256, c, 0u), y);
  }
}

// Slice-by-4 lookups on the 8-replica layout above.
struct LaneTabs4 {
  uint32_t t[4];  // v_perm byte 0 of the lookup address: table and replica bits
  uint32_t s[4];  // v_perm selector: which byte of the state indexes lookup i
};

struct TabsS4 {
  typedef LaneTabs4 LT;
  __device__ static __forceinline__ LT lane(uint32_t u) {
    const uint32_t r = u & 7u, q = (u >> 3) & 3u;
    LT lt;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t k = (q + i) & 3u;  // table T_k, indexed by byte 3 - k of the state
      lt.t[i] = (k * 8u + r) << 2;
      lt.s[i] = sel_byte(3u - k);
    }
    return lt;
  }
  __device__ static __forceinline__ uint32_t step(const char* lds, const LT& lt, uint32_t x, uint32_t w) {
    const uint32_t a0 = __builtin_amdgcn_perm(lt.t[0], x, lt.s[0]);
    const uint32_t a1 = __builtin_amdgcn_perm(lt.t[1], x, lt.s[1]);
    const uint32_t a2 = __builtin_amdgcn_perm(lt.t[2], x, lt.s[2]);
    const uint32_t a3 = __builtin_amdgcn_perm(lt.t[3], x, lt.s[3]);
    return xor3(xor3(lds_u32(lds, a0), lds_u32(lds, a1), lds_u32(lds, a2)), lds_u32(lds, a3), w);
  }
  // four independent chains stepped together: all 16 lookups are issued before the first result
  // is consumed (left to itself the scheduler issues them in groups of 4-8 and waits for each
  // group, one LDS round trip per group)
  __device__ static __forceinline__ void step4(const char* lds, const LT& lt, uint32_t (&x)[4], const uint32_t (&w)[4]) {
    uint32_t a[16], v[16];
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c)
#pragma unroll
      for (uint32_t i = 0; i < 4; ++i) a[4 * c + i] = __builtin_amdgcn_perm(lt.t[i], x[c], lt.s[i]);
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) v[j] = lds_u32(lds, a[j]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c) x[c] = xor3(xor3(v[4 * c], v[4 * c + 1], v[4 * c + 2]), v[4 * c + 3], w[c]);
  }
  // three chains stepped together (the 27-word parts' steps before chain D starts): all 12
  // lookups issued before the first result is consumed, as in step4
  __device__ static __forceinline__ void step3(const char* lds, const LT& lt, uint32_t (&x)[3], const uint32_t (&w)[3]) {
    uint32_t a[12], v[12];
#pragma unroll
    for (uint32_t c = 0; c < 3; ++c)
#pragma unroll
      for (uint32_t i = 0; i < 4; ++i) a[4 * c + i] = __builtin_amdgcn_perm(lt.t[i], x[c], lt.s[i]);
#pragma unroll
    for (uint32_t j = 0; j < 12; ++j) v[j] = lds_u32(lds, a[j]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (uint32_t c = 0; c < 3; ++c) x[c] = xor3(xor3(v[4 * c], v[4 * c + 1], v[4 * c + 2]), v[4 * c + 3], w[c]);
  }
  // two chains stepped together (diagnostics MODE 51: a part as two chains): 8 lookups issued together
  __device__ static __forceinline__ void step2(const char* lds, const LT& lt, uint32_t (&x)[2], const uint32_t (&w)[2]) {
    uint32_t a[8], v[8];
#pragma unroll
    for (uint32_t c = 0; c < 2; ++c)
#pragma unroll
      for (uint32_t i = 0; i < 4; ++i) a[4 * c + i] = __builtin_amdgcn_perm(lt.t[i], x[c], lt.s[i]);
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) v[j] = lds_u32(lds, a[j]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (uint32_t c = 0; c < 2; ++c) x[c] = xor3(xor3(v[4 * c], v[4 * c + 1], v[4 * c + 2]), v[4 * c + 3], w[c]);
  }
  __device__ static __forceinline__ void stage(char* lds, const uint32_t* __restrict__ tabs) {
    // T0..T3 x 8 replicas: 256 entries x 4 tables x 2 quads of 16 B; quad i at b<<8 | k<<5 | h<<4
    for (uint32_t i = threadIdx.x; i < 2048u; i += blockDim.x) {
      const uint32_t b = i >> 3, k = (i >> 1) & 3u, h = i & 1u;
      const uint32_t v = tabs[k * 256u + b];  // tabs: T0[256] T1[256] T2[256] T3[256]
      *reinterpret_cast<u32x4*>(lds + ((b << 8) | (k << 5) | (h << 4))) = u32x4{v, v, v, v};
    }
  }
};

template <uint32_t kOpSet>
__device__ __forceinline__ void stage_ops_span(char* lds, const uint32_t* __restrict__ tabs) {
  // slot s, sub-table j, entry b at b<<8 | 128 | (((b >> 2) ^ (4s + j)) & 31) << 2; sources: catalog
  // entries 1 (32), 2 (64), 4 (256), 6 (1024), then the class's part operators (132, 264, 528 or
  // 108, 216, 432); slot 0 = the class's 3-part operator (396 or 324)
  for (uint32_t i = threadIdx.x; i < 8u * 1024u; i += blockDim.x) {
    const uint32_t slot = i >> 10, j = (i >> 8) & 3u, b = i & 255u;
    const uint32_t src = slot == 0u  ? PDB_SPANOP_OFF + (kOpSet == 0u ? 6u : 7u) * 1024u
                         : slot < 5u ? 1024u + (slot < 3u ? slot : (slot == 3u ? 4u : 6u)) * 1024u
                                     : PDB_SPANOP_OFF + (slot - 5u + kOpSet) * 1024u;
    *reinterpret_cast<uint32_t*>(lds + ((b << 8) | 128u | ((((b >> 2) ^ (4u * slot + j)) & 31u) << 2))) = tabs[src + j * 256u + b];
  }
}

// Whole-wave hash of one record of any length from global memory (Value() seed): the slow path of
// crc_sized_kernel (slow_finish) on this kernel's operator layout.  Rows of 1 KiB: lane u hashes the
// 16-B pieces at 16u + 1024k of the record front-padded with zeros to whole KiB (masked below p, U[z]
// on the piece holding p), Horner-folded with shift 1024; then a 6-level tree (16 .. 512).
template <class TP>
__device__ __forceinline__ uint32_t span_chain16(const char* lds, const typename TP::LT& lt, uint32_t start,
                                                 const uint32_t (&w)[4]) {
  uint32_t x = start ^ w[0];
  x = TP::step(lds, lt, x, w[1]);
  x = TP::step(lds, lt, x, w[2]);
  x = TP::step(lds, lt, x, w[3]);
  return TP::step(lds, lt, x, 0u);
}

template <class TP>
__device__ __forceinline__ uint32_t span_slow_record(const char* lds, const typename TP::LT& lt, uint32_t u, uint32_t ureg,
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
    acc = span_op_x(lds, kOp1024, acc, span_chain16<TP>(lds, lt, start, w));  // acc = shift1024(acc) ^ row
  }
  // tree over 64 lanes, 16 B apart: shift 16 << k between partners at distance 2^k
  uint32_t y;
  y = __builtin_amdgcn_update_dpp(0u, acc, 0x101, 0xF, 0xF, false);  // row_shl:1
  if ((u & 1u) == 0) acc = span_shift_x<TP>(lds, lt, 0, acc, y);
  y = __builtin_amdgcn_update_dpp(0u, acc, 0x102, 0xF, 0xF, false);
  if ((u & 3u) == 0) acc = span_shift_x<TP>(lds, lt, 1, acc, y);
  y = __builtin_amdgcn_update_dpp(0u, acc, 0x104, 0xF, 0xF, false);
  if ((u & 7u) == 0) acc = span_shift_x<TP>(lds, lt, 2, acc, y);
  y = __builtin_amdgcn_update_dpp(0u, acc, 0x108, 0xF, 0xF, false);
  if ((u & 15u) == 0) acc = span_shift_x<TP>(lds, lt, 3, acc, y);
  y = __builtin_amdgcn_ds_swizzle(acc, 0x401F);  // lane ^ 16
  if ((u & 31u) == 0) acc = span_shift_x<TP>(lds, lt, 4, acc, y);
  y = __builtin_amdgcn_readlane(acc, 32);
  if (u == 0) acc = span_shift_x<TP>(lds, lt, 5, acc, y);
  return __builtin_amdgcn_readfirstlane(acc);
}

// ---- items ---------------------------------------------------------------------------------------
// A batch is 64 consecutive records (lane r of the batch registers: record 64 * batch + r).  Its
// in-class records are hashed by items: runs of up to G = floor(64 / k) consecutive records, each
// record on k consecutive lanes (lane u: record slot u / k, part c = u % k).  Counted from the
// record's END, part c covers P = kPart words ending 4 P c bytes before the end, as two chains:
// upper its last 2 LC = 16 words, lower the LC + LD before them; part k - 1's lower chain (the head)
// also runs on to the record's start.  Odd parts put the k lanes of a record on k different LDS
// banks at every step (128-B parts would put them all on one).  The chains of an item run in lock
// step: the head chain alone for lim = max(0, nw - P (k - 1) - 3 LC - LD) steps, then N2 =
// max(2 LC, LC + LD) steps in which a chain works from step N2 - len on (the upper chain's first
// word is just loaded: its state starts at 0).  Folds: per lane Q = shift(lower, 64) ^ upper, then
// across the k lanes of a record shift(Q[c + m], 4 P m) ^ Q[c] for m = 1, 2, 4.  (Round 5 hashed a
// part as four chains A, B, C of LC words and D of LD, folded as shift(shift(D, 32) ^ C, 64) ^
// shift(B, 32) ^ A: three operator applications per lane instead of one; MODE 52 keeps that form.)
// k per batch minimises steps per batch for its longest in-class record.
constexpr uint32_t kNoRec = 0x3FFFFFFFu;

struct LaneSpanGeom {
  uint32_t k;      // lanes per record
  uint32_t g;      // records per item: floor(64 / k)
  uint32_t magic;  // ceil(65536 / k): u / k = (u * magic) >> 16 for u < 64
  uint32_t iters;  // lock-step steps per item: lim + NI
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

// OR over the wave of a 32-bit value; every lane must be active
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
  v |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0xB1, 0xF, 0xF, false));
  v |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x4E, 0xF, 0xF, false));
  v |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x141, 0xF, 0xF, false));
  v |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x140, 0xF, 0xF, false));
  return (__builtin_amdgcn_readlane(v, 0) | __builtin_amdgcn_readlane(v, 16)) |
         (__builtin_amdgcn_readlane(v, 32) | __builtin_amdgcn_readlane(v, 48));
}

// inclusive prefix sum over the wave's lanes (lane u: v_0 + .. + v_u); every lane must be active
__device__ __forceinline__ uint32_t wave_incl_add_u32(uint32_t v, uint32_t u) {
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x111, 0xF, 0xF, false));  // row_shr:1
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x112, 0xF, 0xF, false));  // row_shr:2
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x114, 0xF, 0xF, false));  // row_shr:4
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x118, 0xF, 0xF, false));  // row_shr:8
  const uint32_t r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31);
  const uint32_t r2 = __builtin_amdgcn_readlane(v, 47);
  const uint32_t row = u >> 4;
  return v + (row >= 1u ? r0 : 0u) + (row >= 2u ? r1 : 0u) + (row >= 3u ? r2 : 0u);
}

// k for a batch whose longest in-class record has nw words: the fewest chain steps per batch,
// items per batch x steps per item, with the records an item can hold: G = floor(64 / k), and
// what fits a staging region at ~4 nw + 8 bytes a record
template <uint32_t KMAX, class ST, uint32_t kNIx = ST::kNI>
__device__ __forceinline__ LaneSpanGeom span_pick(uint32_t nw) {
  const float fit = static_cast<float>(ST::kUsable) * __builtin_amdgcn_rcpf(static_cast<float>(4u * nw + 8u));
  uint32_t gfit = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(fit)));
  gfit = gfit ? gfit : 1u;
  LaneSpanGeom best{1u, 64u, 65536u, kNIx};
  uint32_t best_cost = ~0u;
#pragma unroll
  for (uint32_t k = 1; k <= KMAX; ++k) {
    const uint32_t g = 64u / k;
    const uint32_t geff = g < gfit ? g : gfit;
    const int32_t h = static_cast<int32_t>(nw) - static_cast<int32_t>((k - 1u) * ST::kPart + 3u * ST::kLC + ST::kLD);
    const uint32_t it = kNIx + (h > 0 ? static_cast<uint32_t>(h) : 0u);  // lim + NI
    const uint32_t items = (64u + geff - 1u) / geff;
    if (items * it < best_cost) {
      best = LaneSpanGeom{k, g, (65536u + k - 1u) / k, it};
      best_cost = items * it;
    }
  }
  return best;
}

struct SpanItem {
  uint64_t r0;      // records r0 + r (the unit's first record)
  uintptr_t lo;     // 16-B aligned global address of region byte 0
  uint32_t hi;      // local end: max over the item's records (0: nothing to hash)
  uint32_t k, iters;            // k: lanes per record (var: the most any record of the item takes)
  bool valid;
  bool var;                     // per-record lane counts (mixed sizes; open_batch)
  uint32_t r;                   // per lane: record slot in the batch
  uint32_t cw;                  // per lane: part c; kVar classes pack (one VGPR per item in flight)
                                // c (bits 0-3) and the record's parts after it, kl - 1 - c (4-7),
                                // + the item's records (8-14) and first record in its batch of 64 (16-21) in MODE 18
  uint32_t p_loc, e_loc, pre;  // per lane: local start (kNoRec: no record), local end, sink word
};

// MODE (diagnostics only, libpdb_crc32c_diag.so): 0 the product; 1 loads and staging without the
// hash; 2 the hash over whatever the region holds, without the loads; 3 neither (the per-item
// bookkeeping alone); 17 the batch-uniform k only (no per-record lanes for mixed sizes); 18 the
// item geometry instead of the CRC (first record << 24 | records << 16 | lane << 8 | lanes << 4 |
// per-record mode); 40 / 41 / 42 = 0 / 1 / 2 with per-wave clock stamps (a Sink with a `stamps`
// array); 52 the four-chain parts of round 5 (exact), also the form the pricing modes 43-48 price.  The
// round-2..4 A/B forms that lost are recorded in DESIGN.md's appendix and were removed in round 5.
// TP: the table scheme.
// kDyn: false = static batches wv + k W (diagnostics).
// kMixed (PDB_CRC_SIZE_MIXED): per-record lane counts where a batch's records vary (open_batch).
template <class Src, class Sink, uint32_t MAXN, int MODE = 0, class TP = TabsS4, bool kDyn = true, bool kMixed = false>
__global__ __launch_bounds__((SpanStage<MAXN>::kWaves * 64)) void crc_lanespan_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                                       uint64_t nblk, Sink sink) {
  constexpr uint32_t kSpanWaves = SpanStage<MAXN>::kWaves, kSpanJ = SpanStage<MAXN>::kJ;
  constexpr uint32_t kSpanRegion = SpanStage<MAXN>::kRegion, kSpanUsable = SpanStage<MAXN>::kUsable;
  typedef SpanStage<MAXN> ST;
  constexpr uint32_t LC = ST::kLC, LD = ST::kLD, NI = ST::kNI, PART = ST::kPart;
  // A part as TWO chains (round 6): upper = its last 2 LC words, lower = the LC + LD before them (the
  // head chain), folded by ONE shift-64 operator instead of the three of four chains (A..D: S32, S32,
  // S64 -- value-dependent, bank-conflicted single-copy operator lookups), in N2 lock-step steps
  // instead of NI with 8 lookups in flight per step instead of 16: +0.3 / +0.8 / +1.9 / +0.3 % on
  // wal100 / wal400 / wal1000 / wal, +0.5 / +1.3 % on random 300-500- / 64-1000-B records, both orders
  // (tools/ab_span.py, profiles/r06/two_chains/).  MODE 52 (diagnostics, exact) keeps the four-chain
  // form; the pricing modes 43-48 price that form.
  constexpr bool k2 = MODE != 52 && !(MODE >= 43 && MODE <= 48);
  constexpr uint32_t N2 = 2u * LC > LC + LD ? 2u * LC : LC + LD;
  constexpr uint32_t NIH = k2 ? N2 : NI;  // lock-step steps of a part in this mode
  static_assert(MAXN + 32u <= kSpanUsable, "a record of the class must fit a region");
  // k parts cover MAXN: 2, 5, 8 (a longer class -- diagnostics 1152 -- stays at 8 lanes and runs
  // the head chain alone for the rest)
  constexpr uint32_t KMAX = (MAXN / 4u + PART) / PART > 8u ? 8u : (MAXN / 4u + PART) / PART;
  static_assert(KMAX >= 1 && KMAX <= 8, "tree folds for up to 8 lanes per record");
  // per-record lanes for mixed sizes (open_batch): the 257..512- and 513..1023-B classes, whose
  // records take 3..5 and 4..8 lanes; the 9-KiB-region classes (<= 256 B: 1-2 lanes; 1024..1152 B:
  // always 8) have no registers to spare for it (their 2 x 9 staging chunks in flight), nor has the
  // verify form (an expected word per item in flight: it spilled 24-28 B per lane with it)
  constexpr bool kVar = kMixed && MODE != 17 && (MAXN == 512u || MAXN == 1023u) && !__is_same(Sink, VerifySink);
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  TP::stage(lds, tabs);
  stage_ops_span<ST::kOpSet>(lds, tabs);
  const uint32_t u = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ureg = tabs[PDB_UNSHIFT_OFF + (u & 15u)];
  uint64_t t_start = 0;
  uint64_t c_start = 0;
  constexpr bool kClk = MODE >= 40 && MODE <= 42;  // diagnostics: shader-clock stamps (tools/span_clock.py)
  if constexpr (kClk) t_start = wall_clock64();
  if constexpr (kClk) c_start = clock64();
  // Work units (first record r0, records cnt <= 64): the workgroup owns batches [g nbat / G,
  // (g + 1) nbat / G) and its waves take them from an LDS counter; the range's last kWaves batches
  // are split in kS units of 64 / kS records (16: one item of the 512 class, two of the 1023 / 1152
  // classes; the <= 256 class keeps whole batches, one or two items each), so the waves run out of
  // work within about an item of each other instead of a batch (~40 us on 1000-B records): +1.3-1.5 %
  // on wal400 / wal1000 (profiles/r05/queues/).  Each wave holds one ticket in flight (the unit after
  // the one whose descriptors are in flight), so the LDS atomic's latency never waits in front of a
  // load.  (Device-wide queues -- for all the work, or a pool for the tail -- measured 1-16 % slower:
  // profiles/r05/queues/README.md.)  kDyn false (diagnostics): static batches wv + k W.
  // the counter: the last 16 B of the last wave's region, which no item ever uses (spans end by
  // kUsable) and to_lds skips
  uint32_t* ctr = reinterpret_cast<uint32_t*>(lds + kSpanStageBase + kSpanWaves * kSpanRegion - 16u);
  if (kDyn && threadIdx.x == 0) *ctr = kSpanWaves;  // ticket wv is each wave's first
  __syncthreads();
  const typename TP::LT lt = TP::lane(u);
  char* region = lds + kSpanStageBase + wv * kSpanRegion;
  const uintptr_t dummy = reinterpret_cast<uintptr_t>(tabs);  // >= 4 KiB + 256 B of valid bytes
  const uint64_t nbat = (nblk + 63u) >> 6;
  const uint64_t W = static_cast<uint64_t>(gridDim.x) * kSpanWaves;
  constexpr uint32_t kS = MAXN <= 256u ? 1u : 4u;  // units per split batch
  uint32_t tick = wv;  // lane 0: the ticket in flight
  uint64_t sbat = static_cast<uint64_t>(blockIdx.x) * kSpanWaves + wv;  // kDyn false: the next batch
  const uint64_t g_lo = nbat * blockIdx.x / gridDim.x, g_end = nbat * (blockIdx.x + 1) / gridDim.x;
  auto unit_of_batch = [&](uint64_t b, uint64_t& r0, uint32_t& cnt) {
    r0 = b << 6;
    cnt = static_cast<uint32_t>(nblk - r0 < 64u ? nblk - r0 : 64u);
  };
  // ticket t of the workgroup's range: false when exhausted; cnt 0 = an empty unit past nblk
  auto decode = [&](uint32_t t, uint64_t& r0, uint32_t& cnt) -> bool {
    const uint64_t n = g_end - g_lo;
    const uint64_t R = kS == 1u ? 0u : (n < kSpanWaves ? n : kSpanWaves), F = n - R;
    if (t < F) {
      unit_of_batch(g_lo + t, r0, cnt);
      return true;
    }
    const uint64_t q = t - F;
    if (q >= kS * R) return false;
    r0 = ((g_lo + F + q / kS) << 6) + (q % kS) * (64u / kS);
    cnt = r0 >= nblk ? 0u : static_cast<uint32_t>(nblk - r0 < 64u / kS ? nblk - r0 : 64u / kS);
    return true;
  };
  // the next unit (false: no work left): decode the ticket in flight, put the following one in flight
  auto acquire = [&](uint64_t& r0, uint32_t& cnt) -> bool {
    if constexpr (!kDyn) {
      if (sbat >= nbat) return false;
      unit_of_batch(sbat, r0, cnt);
      sbat += W;
      return true;
    } else {
      for (;;) {
        const uint32_t t = __builtin_amdgcn_readfirstlane(tick);
        if (!decode(t, r0, cnt)) return false;
        if (u == 0) tick = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cnt) return true;  // (else an empty unit, the last batch's: the next ticket)
      }
    }
  };
  uint64_t nx_r0 = 0;  // the next unit (its descriptors in flight)
  uint32_t nx_cnt = 0;
  bool nx_ok = acquire(nx_r0, nx_cnt);
  auto idx = [&](uint64_t r0, uint32_t cnt) -> uint64_t { return r0 + (u < cnt ? u : cnt - 1u); };
  // the next unit's descriptors and sink words, in flight; reloaded by every next_item call (the
  // same address when no unit was opened) so no load is ever consumed right after it is issued
  typename Src::Raw raw_next = src.load_cached(idx(nx_r0, nx_ok ? nx_cnt : 1u));
  uint32_t pre_next = SinkOps<Sink>::pre(sink, idx(nx_r0, nx_ok ? nx_cnt : 1u), BlkDesc{nullptr, 0u, 0u});
  uint64_t b_r0 = 0;  // the current unit
  uint32_t b_cnt = 0;
  bool have_batch = false;
  uintptr_t bp = 0;      // per lane: record start
  uint32_t bn = 0;       // per lane: record length
  bool bfast = false;    // per lane: in the class (hashed from LDS)
  uint32_t bpre = 0;     // per lane: the sink's word
  uint64_t bfastm = 0;   // in-class records
  uint64_t bbroken = 0;  // bit r: records r and r + 1 may not share an item
  uint64_t bswap = 0;    // k = 4: bit 16 r + 15 = row r's item splits its records into halves as C (next_item)
  bool bvar = false;     // mixed sizes: record r on bkr lanes (not the batch-uniform k)
  uint32_t bkw = 0;      // per lane: the record's lanes kr = ceil(words / PART) <= KMAX (bits 0-3; 0: not in
                         // the class) | the inclusive prefix sum of kr over the batch (bits 4..)
  uint32_t bkmax = 1, biters_v = NIH;
  uint32_t bcursor = 64;
  LaneSpanGeom bg{1u, 64u, 65536u, NIH};

  // make the prefetched batch current; records outside the class are hashed here by the whole
  // wave (rare: their loads wait behind the items in flight)
  auto open_batch = [&]() -> bool {
    if (!nx_ok) return false;
    keep_alive(raw_next);
    const BlkDesc d = src.lane(raw_next);
    bpre = pre_next;
    b_r0 = nx_r0;
    b_cnt = nx_cnt;
    nx_ok = acquire(nx_r0, nx_cnt);
    const bool valid = u < b_cnt;
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
      const uint32_t rs = span_slow_record<TP>(lds, lt, u, ureg, sp, sn);
      if (u == 0)
        SinkOps<Sink>::put(sink, b_r0 + k, rs, BlkDesc{reinterpret_cast<const uint8_t*>(sp), sn, 0xFFFFFFFFu},
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
    // the lanes cover a record's dwords after its p-word (the hash takes the p-word on the head lane
    // either way): nw = dwords of [p, p + n) on the grid - 1 <= ceil(n / 4)
    const uint32_t nwl = ((plo & 3u) + bn + 3u) >> 2;
    const uint32_t nw = wave_max_u32(bfast ? (nwl > 1u ? nwl - 1u : 1u) : 0u);
    bg = span_pick<KMAX, ST, NIH>(nw ? nw : 1u);
    bcursor = 0;
    // Mixed sizes: the batch-uniform k is set by the longest record, so a short record's lanes
    // would hash padding.  Per-record lanes instead: record r on kr = ceil(words / PART) lanes
    // (<= KMAX; the head chain runs on past KMAX parts), an item's records on consecutive lane
    // ranges (exclusive prefix sums of kr); taken when the item-count model says it pays:
    // items x (steps + 4), items bounded by the lanes (sum kr / 64) and the staging span.
    bvar = false;
    if constexpr (kVar) {
      const uint32_t nwr = nwl > 1u ? nwl - 1u : 1u;
      const uint32_t kq = (nwr + PART - 1u) / PART;
      const uint32_t bkr = bfast ? (kq < KMAX ? (kq ? kq : 1u) : KMAX) : 0u;
      bkw = bkr;
      // the longest record's lanes from the batch's longest record (nw, above); records on fewer
      // lanes save at most kmx - 1 each: fewer than 32 lanes saved cannot drop an item (a log of
      // equal records with its block-end fragments) -- no scan, no extra cost on such batches
      const uint32_t kq1 = (nw + PART - 1u) / PART;
      const uint32_t kmx = kq1 < KMAX ? (kq1 ? kq1 : 1u) : KMAX;
      const uint32_t nsmall = static_cast<uint32_t>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(bfast && bkr < kmx)));
      if (nsmall * (kmx - 1u) >= 32u) {
        const uint32_t bks = wave_incl_add_u32(bkr, u);
        bkw = bkr | (bks << 4);
        const uint32_t sumk = __builtin_amdgcn_readlane(bks, 63);
        const uint32_t limr = bfast && nwr > bkr * PART ? nwr - bkr * PART : 0u;
        const uint32_t iv = NIH + wave_max_u32(limr);
        const uint32_t f0 = static_cast<uint32_t>(__builtin_ctzll(bfastm)), f1 = 63u - static_cast<uint32_t>(__builtin_clzll(bfastm));
        const uint32_t span = (__builtin_amdgcn_readlane(plo, f1) + __builtin_amdgcn_readlane(bn, f1)) -
                              (__builtin_amdgcn_readlane(plo, f0) & ~15u);
        const uint32_t by_span = (span + kSpanUsable - 1u) / kSpanUsable;
        const uint32_t nfast = static_cast<uint32_t>(__builtin_popcountll(bfastm));
        const uint32_t iu = max((nfast + bg.g - 1u) / bg.g, by_span);
        const uint32_t ivn = max((sumk + 63u) >> 6, by_span);
        if (ivn * (iv + 4u) < iu * (bg.iters + 4u)) {
          bvar = true;
          bkmax = kmx;
          biters_v = iv;
        }
      }
    }
    // Bank spread of the staging reads (k = 4: 4 lanes per record, 8 records per 32-lane half).
    // Every lane reads its words at (part end) / 4 + t, so the LDS banks of a read instruction are
    // the half's 32 part-end dword residues mod 32, the same at every step; equal-sized records can
    // pile onto a few banks (431-B records: 4-way conflicts on every staging read).  For each row
    // of 16 records (one full item), count the distinct banks of the two ways of splitting it into
    // halves -- records 0-7 | 8-15 (A) or 0-3, 8-11 | 4-7, 12-15 (C) -- and keep the better (bit
    // 16 r + 15 of bswap: row r takes C).
    bswap = 0;
    if (bg.k == 4u && !bvar) {
      // the lane's 4 part-end residues: ew, ew - P, ew - 2P, ew - 3P (mod 32) = a rotation of one
      // constant mask; quad-OR, then per row the two splits' distinct-bank counts by DPP in lane
      // 16 r + 15 (row_shr 4: quads 0|1 and 2|3; row_shr 8: quads 0|2 and 1|3)
      constexpr uint32_t kM0 = (1u << 0) | (1u << ((32u - ST::kPart % 32u) % 32u)) |
                               (1u << ((64u - 2u * ST::kPart % 32u) % 32u)) | (1u << ((96u - 3u * ST::kPart % 32u) % 32u));
      const uint32_t ew = ((plo + bn + 3u) >> 2) & 31u;
      uint32_t msk = bfast ? __builtin_amdgcn_alignbit(kM0, kM0, (32u - ew) & 31u) : 0u;
      msk |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(msk), 0x111, 0xF, 0xF, false));
      msk |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(msk), 0x112, 0xF, 0xF, false));
      const uint32_t pa = __builtin_popcount(msk | static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(msk), 0x114, 0xF, 0xF, false)));
      const uint32_t pc = __builtin_popcount(msk | static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(msk), 0x118, 0xF, 0xF, false)));
      const uint32_t da = pa + static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(pa), 0x118, 0xF, 0xF, false));
      const uint32_t dc = pc + static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(pc), 0x114, 0xF, 0xF, false));
      bswap = __builtin_amdgcn_ballot_w64((u & 15u) == 15u && dc > da);
    }
    return true;
  };

  // the next item: the next run of in-class records of the current batch (or of the next batch);
  // every field is set on every path (a partially written item ends up in scratch)
  auto next_item = [&](bool want) -> SpanItem {
    SpanItem it;
    it.valid = false;
    it.r0 = b_r0;
    it.lo = dummy;
    it.hi = 0;
    it.k = bg.k;
    it.iters = bg.iters;
    it.var = false;
    it.r = u;
    it.cw = 0;
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
    raw_next = src.load_cached(nx_ok ? idx(nx_r0, nx_cnt) : idx(b_r0, b_cnt));
    pre_next = SinkOps<Sink>::pre(sink, nx_ok ? idx(nx_r0, nx_cnt) : idx(b_r0, b_cnt), BlkDesc{nullptr, 0u, 0u});
    it.valid = true;
    it.r0 = b_r0;
    it.k = bvar ? bkmax : bg.k;
    it.iters = bvar ? biters_v : bg.iters;
    it.var = kVar && bvar;
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
    const uint32_t lo32 = static_cast<uint32_t>(lo);
    // within a linked run the records ascend from lo: 32-bit offsets (lanes outside it are cut by m1)
    const uint64_t over = __builtin_amdgcn_ballot_w64(bfast && u >= g0 && plo + bn - lo32 > kSpanUsable) >> g0;
    const uint32_t m2 = over ? static_cast<uint32_t>(__builtin_ctzll(over)) : 64u;
    if (kVar && bvar) {
      // records g0.. on consecutive lane ranges: lanes of record r = [S(r) - kr - base, S(r) - base)
      const uint32_t bkr = bkw & 15u, bks = bkw >> 4;
      const uint32_t base = __builtin_amdgcn_readlane(bks, g0) - __builtin_amdgcn_readlane(bkr, g0);
      const uint64_t fit = ~(__builtin_amdgcn_ballot_w64(u >= g0 && bks - base <= 64u) >> g0);
      const uint32_t m3 = fit ? static_cast<uint32_t>(__builtin_ctzll(fit)) : 64u - g0;
      const uint32_t m = min(min(m1, m2), m3);
      bcursor = g0 + m;
      it.lo = lo;
      // the start lanes of the item's records as one 64-bit mask; lane u's record is the last
      // start at or below u
      const bool inr = u >= g0 && u < g0 + m;
      const uint32_t st = bks - bkr - base;  // (lanes in range: < 64)
      const uint32_t mlo = wave_or_u32(inr && st < 32u ? 1u << (st & 31u) : 0u);
      const uint32_t mhi = wave_or_u32(inr && st >= 32u ? 1u << (st & 31u) : 0u);
      const uint64_t M = (static_cast<uint64_t>(mhi) << 32) | mlo;
      const uint32_t used = __builtin_amdgcn_readlane(bks, g0 + m - 1u) - base;
      const uint64_t below = M & (u == 63u ? ~0ull : ((2ull << u) - 1ull));
      const bool act = u < used && below != 0;
      const uint32_t rel = static_cast<uint32_t>(__builtin_popcountll(below)) - 1u;
      const uint32_t s0 = 63u - static_cast<uint32_t>(__builtin_clzll(below | 1ull));
      const uint32_t rl = act ? g0 + rel : u;
      // (every bpermute with all lanes active: a source lane outside EXEC reads as 0)
      const uint32_t pr = __shfl(plo, rl, 64), nr = __shfl(bn, rl, 64);
      const uint32_t kr = static_cast<uint32_t>(__shfl(static_cast<int>(bkr), static_cast<int>(rl), 64));
      it.pre = __shfl(bpre, rl, 64);
      const uint32_t c = act ? u - s0 : 0u;
      it.cw = c | ((act ? kr - 1u - c : 0u) << 4) | (MODE == 18 ? (m << 8) | ((g0 + static_cast<uint32_t>(b_r0 & 63u)) << 16) : 0u);
      it.r = rl;
      it.p_loc = act ? pr - lo32 : kNoRec;
      it.e_loc = act ? pr + nr - lo32 : 0u;
      it.hi = wave_max_u32(it.e_loc);
      return it;
    }
    const uint32_t m = min(min(bg.g, m1), m2);
    bcursor = g0 + m;
    it.lo = lo;
    if (bg.k == 1u && g0 == 0u) {  // the common case: lane u hashes record u
      const bool act = u < m;
      it.r = u;
      it.cw = (kVar && MODE == 18) ? (m << 8) | ((g0 + static_cast<uint32_t>(b_r0 & 63u)) << 16) : 0u;
      it.pre = bpre;
      it.p_loc = act ? plo - lo32 : kNoRec;
      it.e_loc = act ? plo + bn - lo32 : 0u;
    } else {
      uint32_t slot = (u * bg.magic) >> 16;
      const uint32_t c = u - slot * bg.k;
      bool act;
      uint32_t rl, pr = 0, nr = 0;
      // k = 4, an item of 16 records aligned on a row of the batch: open_batch chose how to split
      // them into the two 32-lane halves (bswap)
      if (bg.k == 4u && (g0 & 15u) == 0 && m == 16u && ((bswap >> (g0 | 15u)) & 1u))
        slot = (slot & 3u) | ((slot & 4u) << 1) | ((slot & 8u) >> 1);  // slot bits 2 and 3 exchanged
      act = slot < m;
      rl = act ? g0 + slot : u;
      pr = __shfl(plo, rl, 64);
      nr = __shfl(bn, rl, 64);
      it.pre = __shfl(bpre, rl, 64);
      it.r = rl;
      it.cw = kVar ? c | ((bg.k - 1u - c) << 4) | (MODE == 18 ? (m << 8) | ((g0 + static_cast<uint32_t>(b_r0 & 63u)) << 16) : 0u) : c;
      it.p_loc = act ? pr - lo32 : kNoRec;
      it.e_loc = act ? pr + nr - lo32 : 0u;
    }
    it.hi = wave_max_u32(it.e_loc);
    return it;
  };

  // loads of one item: kSpanJ unconditional 16-B buffer loads (1 KiB contiguous per instruction,
  // non-temporal) from the item's uniform base, the descriptor's range check ending at its last
  // 16-B chunk: chunks past it read as zeros without touching memory (an empty item reads the
  // tables' first 16 B).  32-bit lane offsets, no per-chunk address arithmetic.
  auto issue = [&](u32x4 (&A)[kSpanJ], const SpanItem& it) {
    const uint32_t lo_l = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(it.lo));
    const uint32_t lo_h = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(static_cast<uint64_t>(it.lo) >> 32));
    const uint32_t nb = (MODE == 2 || MODE == 3 || MODE == 42) ? 16u : __builtin_amdgcn_readfirstlane(it.hi ? (it.hi + 15u) & ~15u : 16u);
    void* base = reinterpret_cast<void*>((static_cast<uint64_t>(lo_h) << 32) | lo_l);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, static_cast<int>(nb), 0x00020000);
#pragma unroll
    for (uint32_t j = 0; j < kSpanJ; ++j)
      A[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(1024u * j + 16u * u), 0,
                                                                              2 /* nt */));
  };
  // The region receives the chunks below the item's end + 64 B, the rest are not written (+0.8 % on
  // wal400, +2 % on random 300-500-B records in A/B, profiles/r04/ab/ab_skiptail.log): the hash
  // reads a record's words as dword pairs ending within 4 B past the record's end and the p-word's
  // pair within 8 B past its start, all below hi + 8, so the 64-B margin is never read past.  (The
  // unwritten chunks' loads still complete before their registers are reloaded by the next issue().)
  static_assert(64u >= 8u, "the staged margin covers the hash's read window past hi");
  auto to_lds = [&](const u32x4 (&A)[kSpanJ], const SpanItem& it) {
    const uint32_t nw = __builtin_amdgcn_readfirstlane(it.hi) + 64u;
    if constexpr (MODE == 47) {  // pricing: one store of the chunks' XOR (wrong CRCs by design)
      u32x4 x = A[0];
#pragma unroll
      for (uint32_t j = 1; j < kSpanJ; ++j) x ^= A[j];
      *reinterpret_cast<u32x4*>(region + 16u * u) = x;
      return;
    }
#pragma unroll
    for (uint32_t j = 0; j + 1 < kSpanJ; ++j)
      if (j == 0 || 1024u * j < nw) *reinterpret_cast<u32x4*>(region + 1024u * j + 16u * u) = A[j];
    // the last chunk: its lanes that fall inside the region (all of them for 8-KiB regions), but not
    // the last 16 B of the last region, which hold the counter
    constexpr uint32_t kLast = SpanStage<MAXN>::kLastLanes;
    if (1024u * (kSpanJ - 1u) < nw)
      if (u < kLast && (!kDyn || wv + 1u < kSpanWaves || u != kLast - 1u))
        *reinterpret_cast<u32x4*>(region + 1024u * (kSpanJ - 1u) + 16u * u) = A[kSpanJ - 1u];
  };
  // hash an item staged in the region
  auto hash = [&](const SpanItem& it) {
    if (it.hi == 0 || MODE == 1 || MODE == 3 || MODE == 41) return;
    // chain X (A, B, C, D = 0..3) works from lock-step step F[X] on; its word at step t is the one
    // ending 4 (NI - t) bytes before the chain's end
    constexpr int32_t FABC = static_cast<int32_t>(NI - LC), FD = static_cast<int32_t>(NI - LD);
    const uint32_t k = it.k, lim = it.iters - NIH;
    const int32_t e = static_cast<int32_t>(it.e_loc);
    const int32_t pl = static_cast<int32_t>(it.p_loc);
    const bool act = it.p_loc != kNoRec;
    // part (kVar: packed per lane with the record's parts after it; else from the uniform k)
    const uint32_t pc = kVar ? it.cw & 15u : it.cw;
    // the record's parts after this one: >= m
    auto more = [&](uint32_t m) -> bool { return kVar ? ((it.cw >> 4) & 15u) >= m : pc + m < k; };
    const bool head = kVar ? ((it.cw >> 4) & 15u) == 0u : pc == k - 1u;
    // Words are the region's dwords (the dword grid): the record's last dword holds j = (-e) mod 4
    // bytes past its end, masked to zero (finished by a shift of 4 - j bytes instead of F), and its
    // first dword, the p-word, zp bytes before p, masked with U[zp] injected.  Part c ends at
    // eg - 4 PART c, eg = e rounded up to the grid.
    const int32_t eg = (e + 3) & ~3;
    const uint32_t j = static_cast<uint32_t>(eg - e);
    const uint32_t endm = 0xFFFFFFFFu >> (8u * j);  // the last dword's bytes in the record
    const uint32_t zp = static_cast<uint32_t>(pl) & 3u;  // bytes of the p-word before p
    const uint32_t uz = __shfl(ureg, zp, 64);
    // The p-word (at sp), masked below p with U[z] injected, replaces its chain's state at its
    // step; a chain wholly before p yields 0.
    const int32_t eA = eg - static_cast<int32_t>(4u * PART * pc);
    const int32_t sp = act ? pl - static_cast<int32_t>(zp) : eg - 4;  // (no record: an address in range)
    const uint32_t pw = (lds_u32(region + sp, 0) & (0xFFFFFFFFu << (8u * zp)) & (sp == eg - 4 ? endm : 0xFFFFFFFFu)) ^ uz;
    // the last word of chain A on part 0 (the record's last dword) keeps the record's bytes only
    const uint32_t lastm = pc == 0 ? endm : 0xFFFFFFFFu;
    uint32_t P = 0, ca = 0, cb = 0, cc = 0, cd = 0;
    // (diagnostics, wrong CRCs by design: MODE 43 prices the folds' operator lookups as free, MODE 44
    // as 8 conflict-free lookups each, MODE 45 with no dependence between them (each indexed by
    // chain states, `alt`), MODE 46 the cross-lane operators alone as free)
    auto fold_op = [&](uint32_t slot, uint32_t c, uint32_t y, uint32_t alt) -> uint32_t {
      if constexpr (MODE == 43) return c ^ y;
      if constexpr (MODE == 44) return TP::step(lds, lt, TP::step(lds, lt, c, 0u), y);
      if constexpr (MODE == 45) return span_op_x(lds, slot, alt, y ^ c);
      if constexpr (MODE == 46) if (slot != kOp32 && slot != kOp64) return c ^ y;
      return span_op_x(lds, slot, c, y);
    };
    if constexpr (k2) {
      // two chains: lower word t at dword qd2 + t (t >= FL: C and D, the head chain), upper word t at
      // qd2 + 2 LC + t (t >= FU: B and A), the upper ending at the part's end eA
      constexpr int32_t FU = static_cast<int32_t>(N2 - 2u * LC), FL = static_cast<int32_t>(N2 - LC - LD);
      const int32_t Tu = static_cast<int32_t>(N2) - ((eA - sp) >> 2);  // the p-word's step, upper numbering
      const int32_t Tl = Tu + static_cast<int32_t>(2u * LC);             // and lower numbering
      const int32_t qd2 = (eA - static_cast<int32_t>(4u * N2 + 8u * LC)) >> 2;
      uint32_t qo2 = static_cast<uint32_t>(region - lds) + static_cast<uint32_t>(4 * qd2);
      asm volatile("" : "+v"(qo2));
      auto sread2 = [&](uint32_t off) -> uint32_t { return lds_u32(lds, qo2 + off); };
      uint32_t xl = 0, xu = 0;
      if (lim > 0) {  // the head chain alone (junk on the other lanes, dropped)
        const int32_t tL = Tl - FL + static_cast<int32_t>(lim);  // the p-word's step in it
        const char* q = region + 4 * (qd2 + FL - static_cast<int32_t>(lim));
        xl = tL == -1 ? pw : 0u;
        for (int32_t t = 0; t < static_cast<int32_t>(lim); ++t, q += 4) {
          const uint32_t w = lds_u32(q, 0);
          xl = t == tL ? pw : TP::step(lds, lt, xl, w);
        }
        xl = head ? xl : 0u;
      } else {
        xl = head && Tl == FL - 1 ? pw : 0u;
      }
#pragma unroll
      for (int32_t t = 0; t < static_cast<int32_t>(N2); ++t) {
        const bool uu = t >= FU, ll = t >= FL;  // compile time
        uint32_t wu = 0, wl = 0;
        if (uu) {
          wu = sread2(8u * LC + 4u * t);
          if (t == static_cast<int32_t>(N2) - 1) wu &= lastm;
        }
        if (ll) wl = sread2(4u * t);
        if (uu && t == FU) {  // the upper chain's first word: the state is 0
          xu = wu;
          if (ll) xl = TP::step(lds, lt, xl, wl);
        } else if (uu && ll) {
          uint32_t x2[2] = {xu, xl};
          const uint32_t w2[2] = {wu, wl};
          TP::step2(lds, lt, x2, w2);
          xu = x2[0], xl = x2[1];
        } else if (uu) {
          xu = TP::step(lds, lt, xu, wu);
        } else if (ll) {
          xl = TP::step(lds, lt, xl, wl);
        }
        if (uu) xu = Tu == t ? pw : xu;
        if (ll) xl = Tl == t ? pw : xl;
      }
      const uint32_t cu = Tu < static_cast<int32_t>(N2) ? xu : 0u;
      const uint32_t cl = Tl < static_cast<int32_t>(N2) ? xl : 0u;
      P = span_op_x(lds, kOp64, cl, cu);  // S64(lower) ^ upper
    } else {
      // the p-word's lock-step step in chain A's numbering; T + LC X in chain X's
      const int32_t T = static_cast<int32_t>(NI) - ((eA - sp) >> 2);
      // base of the chains' words: chain X's dword i at q3 + 4 LC (3 - X) + 4 i (word at step t =
      // dword t); below the region for short records (words never used)
      const int32_t qd = (eA - static_cast<int32_t>(4u * NI + 12u * LC)) >> 2;  // q3's dword (region-relative)
      const char* q3 = region + 4 * qd;
      // the chains' reads are addressed as lds + qo + constant with qo opaque to the compiler, so every
      // read takes its constant in the instruction's offset field (left to itself the compiler re-bases
      // them on the highest address and computes each negative offset with a VALU; +1.9-2.1 % on
      // wal400 / wal1000 / wal in A/B, profiles/r04/ab_variants_r04d.log)
      uint32_t qo = static_cast<uint32_t>(region - lds) + static_cast<uint32_t>(4 * qd);
      asm volatile("" : "+v"(qo));
      auto sread = [&](uint32_t off) -> uint32_t { return lds_u32(lds, qo + off); };
      // The p-word may also be the dword just before the head lane's first word (the lanes cover the
      // record's dwords after its p-word: span_pick counts those): the head chain then starts from it.
      uint32_t xd = 0;
      uint32_t xa = 0, xb = 0, xc = 0;
      if (lim > 0) {  // the head chain alone (junk on the other lanes, dropped)
        const int32_t tD = T + static_cast<int32_t>(3u * LC + lim) - FD;  // the p-word's step in it
        const char* q = q3 + 4 * (FD - static_cast<int32_t>(lim));
        xd = tD == -1 ? pw : 0u;
        for (int32_t t = 0; t < static_cast<int32_t>(lim); ++t, q += 4) {
          const uint32_t w = lds_u32(q, 0);
          xd = t == tD ? pw : TP::step(lds, lt, xd, w);
        }
        xd = head ? xd : 0u;
      } else {
        xd = head && T + static_cast<int32_t>(3u * LC) == FD - 1 ? pw : 0u;
      }
      // The chains' words: one ds_read_b32 per word and chain.  (Aligned ds_read_b64 pairs measured
      // 2.5-9 % slower on every WAL row, profiles/r04/ab_pairs.log: the extra live pair registers and
      // selects.)
      // (diagnostics, wrong CRCs by design: MODE 48 prices the chains' words as 16-B reads, one per
      // four words of a chain, at the 16-B-aligned addresses below them)
      const uint32_t qo16 = qo & ~15u;
      u32x4 qa4{}, qb4{}, qc4{}, qd4{};
      auto sread4 = [&](uint32_t off) -> u32x4 { return *reinterpret_cast<const u32x4*>(lds + qo16 + off); };
  #pragma unroll
      for (int32_t t = 0; t < static_cast<int32_t>(NI); ++t) {
        const bool abc = t >= FABC, dd = t >= FD;  // compile time
        uint32_t wa = 0, wb = 0, wc = 0, wd = 0;
        if constexpr (MODE == 48) {
          if (abc) {
            const uint32_t r = static_cast<uint32_t>(t - FABC);
            if ((r & 3u) == 0) qa4 = sread4(12u * LC + 4u * r), qb4 = sread4(8u * LC + 4u * r), qc4 = sread4(4u * LC + 4u * r);
            wa = qa4[r & 3u], wb = qb4[r & 3u], wc = qc4[r & 3u];
          }
          if (dd) {
            const uint32_t r = static_cast<uint32_t>(t - FD);
            if ((r & 3u) == 0) qd4 = sread4(4u * r);
            wd = qd4[r & 3u];
          }
        } else {
          if (abc) {
            wa = sread(12u * LC + 4u * t), wb = sread(8u * LC + 4u * t), wc = sread(4u * LC + 4u * t);
            if (t == static_cast<int32_t>(NI) - 1) wa &= lastm;
          }
          if (dd) wd = sread(4u * t);
        }
        if (abc && t == FABC) {  // the first word: the state is 0
          xa = wa, xb = wb, xc = wc;
          if (dd) xd = TP::step(lds, lt, xd, wd);
        } else if (abc && dd) {
          uint32_t x4[4] = {xa, xb, xc, xd};
          const uint32_t w4[4] = {wa, wb, wc, wd};
          TP::step4(lds, lt, x4, w4);
          xa = x4[0], xb = x4[1], xc = x4[2], xd = x4[3];
        } else if (abc) {
          uint32_t x3[3] = {xa, xb, xc};
          const uint32_t w3[3] = {wa, wb, wc};
          TP::step3(lds, lt, x3, w3);
          xa = x3[0], xb = x3[1], xc = x3[2];
        } else if (dd) {
          xd = TP::step(lds, lt, xd, wd);
        }
        // the p-word replaces its chain's state: branch-free selects on every step (+0.1-3 % over
        // selects bounded by the item's last replacement step, profiles/r04/ab/ab_nog.log)
        if (abc) {
          xa = T == t ? pw : xa;
          xb = T + static_cast<int32_t>(LC) == t ? pw : xb;
          xc = T + static_cast<int32_t>(2u * LC) == t ? pw : xc;
        }
        if (dd) xd = T + static_cast<int32_t>(3u * LC) == t ? pw : xd;
      }
      // Finish.  Chain X's state still holds its last word unshifted, and its bytes end 32 X bytes
      // before the part's end, so the part's raw CRC is F(xA) ^ S32 F(xB) ^ S64 F(xC) ^ S96 F(xD)
      // with F = the table step (shift 4) and S_n = shift n; these maps commute, so it is
      // F(S64(S32(xD) ^ xC) ^ (S32(xB) ^ xA)), and across the k parts of a record
      // F(sum_c S_{4 PART c}(R_c)): ONE table step after the cross-lane fold.
      // A chain whose end is at or before the p-word's start holds no byte of the record.
      const int32_t L = static_cast<int32_t>(NI);
      ca = T < L ? xa : 0u;
      cb = T + static_cast<int32_t>(LC) < L ? xb : 0u;
      cc = T + static_cast<int32_t>(2u * LC) < L ? xc : 0u;
      cd = T + static_cast<int32_t>(3u * LC) < L ? xd : 0u;
      static_assert(LC == 8, "the in-part folds use the 32- and 64-B operators");
      const uint32_t lo2 = fold_op(kOp32, cb, ca, cb);  // S32(B) ^ A
      const uint32_t hi2 = fold_op(kOp32, cd, cc, cd);  // S32(D) ^ C
      P = fold_op(kOp64, hi2, lo2, ca ^ cc);  // S64(hi2) ^ lo2
    }
    if (k > 1u) {
      // the cross-lane fold, pre-shifted per lane: lane c applies shift(R_c, 4 PART (c mod 4)) (slots
      // P1, P2, P3 chosen per lane), the record's quad XOR-reduces, and a record of > 4 parts adds
      // the upper quad's sum shifted by 4 parts (P4) -- one operator level for k <= 4, two for k <= 8
      // (+0.2-1.7 % over the round-3 tree of levels P1, P2, P4, profiles/r04/ab_variants.log).
      // k a power of two: a record's k lanes never straddle a row of 16, so the partner's value
      // comes by DPP row_shl (no LDS round trip); other k by bpermute.
      const bool dpp = (k & (k - 1u)) == 0 && !(kVar && it.var);
      const uint32_t l = pc & 3u;
      const uint32_t slot = l == 1u ? kOpP1 : (l == 2u ? kOpP2 : kOpP3);
      uint32_t Ps;
      if constexpr (MODE >= 43 && MODE <= 46) {
        Ps = fold_op(slot, P, 0u, cb ^ cc);
      } else if constexpr (MODE == 49) {  // (diagnostics: the lookups on the lanes that use them only)
        Ps = P;
        if (l) {
          uint32_t v[4];
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t bb = __builtin_amdgcn_perm(0u, P, 0x0C0C0000u | (j << 8) | j);
            v[j] = lds_u32(lds, (bb & 0xFF7Cu) ^ (128u | ((4u * slot + j) << 2)));
          }
          Ps = xor3(xor3(v[0], v[1], v[2]), v[3], 0u);
        }
      } else {
        uint32_t v[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          const uint32_t bb = __builtin_amdgcn_perm(0u, P, 0x0C0C0000u | (j << 8) | j);
          v[j] = lds_u32(lds, (bb & 0xFF7Cu) ^ (128u | ((4u * slot + j) << 2)));
        }
        Ps = xor3(xor3(v[0], v[1], v[2]), v[3], 0u);
      }
      P = l ? Ps : P;
      uint32_t y = dpp ? static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(P), 0x101, 0xF, 0xF, false))
                       : __shfl_down(P, 1, 64);
      if ((pc & 1u) == 0 && more(1u)) P ^= y;
      if (k > 2u) {
        y = dpp ? static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(P), 0x102, 0xF, 0xF, false))
                : __shfl_down(P, 2, 64);
        if ((pc & 3u) == 0 && more(2u)) P ^= y;
      }
      if (k > 4u) {
        y = dpp ? static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(P), 0x104, 0xF, 0xF, false))
                : __shfl_down(P, 4, 64);
        if ((pc & 7u) == 0 && more(4u)) P = fold_op(kOpP4, y, P, ca ^ cd);
      }
    }
    // F for a last dword of 4 - j record bytes: shift(P, 4 - j bytes) = F(P << 8 j) ^ (P >> 8 (4 - j))
    P = TP::step(lds, lt, P << (8u * j), (P >> (24u - 8u * j)) >> 8);
    if constexpr (MODE == 18)  // diagnostics: the item's first record, records, lane, lanes, mode
      P = ~(((it.cw >> 16) << 24) | (((it.cw >> 8) & 127u) << 16) | (u << 8) | ((kVar ? pc + ((it.cw >> 4) & 15u) + 1u : k) << 4) | (it.var ? 1u : 0u));
    if (pc == 0 && act)
      SinkOps<Sink>::put(sink, it.r0 + it.r, P, BlkDesc{nullptr, 0u, 0xFFFFFFFFu}, it.pre);
  };

  // ---- pipeline: two items in flight while one is hashed ---------------------------------------
  // Loop head: the region holds I0, array B holds I1's loads in flight; only B's loads cross the
  // back edge.  (One item in flight -- half the staging registers, 13 waves of 7 KiB -- measured
  // slower, profiles/r04/ab/ab_onedeep_13waves.log.)
  if (nx_ok) {
    u32x4 A[kSpanJ], B[kSpanJ];
    SpanItem I0 = next_item(true);
    issue(A, I0);
    SpanItem I1 = next_item(I0.valid);
    issue(B, I1);
    to_lds(A, I0);
    while (I0.valid) {
      const SpanItem I2 = next_item(I1.valid);
      issue(A, I2);
      hash(I0);
      if (!I1.valid) break;
      to_lds(B, I1);
      const SpanItem I3 = next_item(I2.valid);
      issue(B, I3);
      hash(I1);
      if (!I2.valid) break;
      to_lds(A, I2);
      I0 = I2;
      I1 = I3;
    }
  }
  if constexpr (kClk) {
    // MODE 40 / 41 / 42 (the product / loads alone / hash alone): [start, end] s_memrealtime (100 MHz)
    // and [start, end] s_memtime (shader clock): the wave's mean clock over its lifetime
    const uint64_t t_end = wall_clock64();
    const uint64_t c_end = clock64();
    if (u == 0) {
      uint64_t* st = sink.stamps + 4u * (static_cast<uint64_t>(blockIdx.x) * kSpanWaves + wv);
      st[0] = t_start;
      st[1] = t_end;
      st[2] = c_start;
      st[3] = c_end;
    }
  }
}

// grid: one wave per batch of 64 records, `waves` per workgroup, at most one workgroup per CU
inline uint32_t grid_span(const LaunchGeom& g, uint64_t nblk, uint32_t waves) {
  const uint64_t want = ((nblk + 63) / 64 + waves - 1) / waves;
  return static_cast<uint32_t>(want < g.grid ? (want ? want : 1) : g.grid);
}

// Records of 1..1152 B by class (the class bounds the lanes per record: 2, 4, 8, 8); longer ones,
// and empty ones, take the whole-wave path.
template <class Src, class Sink, int MODE = 0, class TP = TabsS4, bool kDyn = true>
hipError_t launch_lanespan(const LaunchGeom& g, const uint32_t* d_tables, const Src& src, uint64_t nblk, uint32_t cls,
                           const Sink& sink, hipStream_t s, bool mixed = false) {
  if (cls <= 256u) {
    constexpr uint32_t w = SpanStage<256>::kWaves;
    hipLaunchKernelGGL((crc_lanespan_kernel<Src, Sink, 256, MODE, TP, kDyn>), dim3(grid_span(g, nblk, w)), dim3(w * 64), 0, s,
                       d_tables, src, nblk, sink);
  } else if (cls <= 512u) {
    constexpr uint32_t w = SpanStage<512>::kWaves;
    if (mixed && !__is_same(Sink, VerifySink))
      hipLaunchKernelGGL((crc_lanespan_kernel<Src, Sink, 512, MODE, TP, kDyn, true>), dim3(grid_span(g, nblk, w)), dim3(w * 64),
                         0, s, d_tables, src, nblk, sink);
    else
      hipLaunchKernelGGL((crc_lanespan_kernel<Src, Sink, 512, MODE, TP, kDyn>), dim3(grid_span(g, nblk, w)), dim3(w * 64), 0, s,
                         d_tables, src, nblk, sink);
  } else if (cls <= 1023u) {
    constexpr uint32_t w = SpanStage<1023>::kWaves;
    if (mixed && !__is_same(Sink, VerifySink))
      hipLaunchKernelGGL((crc_lanespan_kernel<Src, Sink, 1023, MODE, TP, kDyn, true>), dim3(grid_span(g, nblk, w)), dim3(w * 64),
                         0, s, d_tables, src, nblk, sink);
    else
      hipLaunchKernelGGL((crc_lanespan_kernel<Src, Sink, 1023, MODE, TP, kDyn>), dim3(grid_span(g, nblk, w)), dim3(w * 64), 0,
                         s, d_tables, src, nblk, sink);
  } else {  // 1024..1152 B (WAL records of ~1-KiB write batches): 8 lanes, the head chain past 1056 B
    constexpr uint32_t w = SpanStage<1152>::kWaves;
    hipLaunchKernelGGL((crc_lanespan_kernel<Src, Sink, 1152, MODE, TP, kDyn>), dim3(grid_span(g, nblk, w)), dim3(w * 64), 0,
                       s, d_tables, src, nblk, sink);
  }
  return hipGetLastError();
}

}  // namespace
}  // namespace pdb
