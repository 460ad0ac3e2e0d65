// crc32c_kernels.hip -- CRC32C (Castagnoli) over batches of independent sstable blocks on
// MI355X (gfx950, CDNA4).  Hand-written HIP; no MFMA (GF(2) byte work is not a contraction).
//
// Replaces the per-block software CRC of the reference: crc32c::Extend -> crc32_software ->
// crc32c_sb8_64_bit (util/crc32c.cc:25-32, 101-103, 585-625), called once per block by
// TableBuilder::WriteRawBlock (table/table_builder.cc:197-199) and ReadBlock
// (table/format.cc:96-98).  Results are bit-identical (tests/golden + oracle parity).
//
// Work decomposition (one wavefront = one block "team"):
//   * a block of n bytes = head (n % 64 bytes, lane 0, serial) + K = n / 64 chunks of 64 B;
//     chunk c belongs to lane c % 64 in round c / 64.  Lane l's 64-B chunk is read with four
//     16-B loads; each lane runs a slice-by-4 chain over its 16 dwords with LDS tables.
//   * between rounds a lane "Horner-shifts" its partial state over the 63 chunks other lanes
//     own (op 6: shift by 4032 B), so one partial per lane covers all its chunks.
//   * a 6-level wavefront tree (shfl_down + shift by 64 << k bytes, ops 0..5) folds the 64
//     partials; a non-multiple-of-64 chunk count is handled by rotating lanes first.
//   * Extend's init enters as lane 0's starting state; Extend = ~state (util/crc32c.cc:27,31).
//
// LDS image (crc32c_math.h): T0..T3 replicated 32x (128 KiB) so each lane reads its own bank,
// + 7 shift operators (28 KiB).  One 1024-thread workgroup per CU stages it once and then
// walks blocks persistently.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_internal.h"
#include "crc32c_math.h"

namespace pdb {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

constexpr uint32_t kThreads = 1024;
constexpr uint32_t kWavesPerWg = kThreads / 64;

// v_perm_b32 selectors: result = [lb.byte0, x.byte j, lb.byte2, 0x00]  (S0 = lb, S1 = x)
constexpr uint32_t sel_byte(uint32_t j) { return 0x0C060004u | (j << 8); }

struct LaneTabs {
  uint32_t t3, t2, t1, t0;  // per-lane LDS address bases of T3..T0 (replica = lane & 31)
};

__device__ __forceinline__ LaneTabs lane_tabs(uint32_t lane) {
  const uint32_t r = (lane & 31u) << 2;
  return LaneTabs{0x10080u | r, 0x10000u | r, 0x00080u | r, r};
}

__device__ __forceinline__ uint32_t lds_u32(const char* lds, uint32_t addr) {
  return *reinterpret_cast<const uint32_t*>(lds + addr);
}

// One slice-by-4 step: c' = shift(c ^ w, 4 bytes).
__device__ __forceinline__ uint32_t step4(const char* lds, const LaneTabs& lt, uint32_t c,
                                          uint32_t w) {
  const uint32_t x = c ^ w;
  const uint32_t a3 = __builtin_amdgcn_perm(lt.t3, x, sel_byte(0));
  const uint32_t a2 = __builtin_amdgcn_perm(lt.t2, x, sel_byte(1));
  const uint32_t a1 = __builtin_amdgcn_perm(lt.t1, x, sel_byte(2));
  const uint32_t a0 = __builtin_amdgcn_perm(lt.t0, x, sel_byte(3));
  return (lds_u32(lds, a3) ^ lds_u32(lds, a2)) ^ (lds_u32(lds, a1) ^ lds_u32(lds, a0));
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // gfx950 v_bitop3_b32: a ^ b ^ c
}

// x' = shift(x, 4 bytes) ^ w_next: one slice-by-4 step whose input is already crc ^ word, with
// the next word folded in (chains carry x = state ^ next data word).
__device__ __forceinline__ uint32_t step4x(const char* lds, const LaneTabs& lt, uint32_t x,
                                           uint32_t wnext) {
  const uint32_t a3 = __builtin_amdgcn_perm(lt.t3, x, sel_byte(0));
  const uint32_t a2 = __builtin_amdgcn_perm(lt.t2, x, sel_byte(1));
  const uint32_t a1 = __builtin_amdgcn_perm(lt.t1, x, sel_byte(2));
  const uint32_t a0 = __builtin_amdgcn_perm(lt.t0, x, sel_byte(3));
  return xor3(xor3(lds_u32(lds, a3), lds_u32(lds, a2), lds_u32(lds, a1)), lds_u32(lds, a0), wnext);
}

// Byte step (util/crc32c.cc:601): c' = T0[(c ^ b) & 0xff] ^ (c >> 8).
__device__ __forceinline__ uint32_t step1(const char* lds, const LaneTabs& lt, uint32_t c,
                                          uint32_t b) {
  return lds_u32(lds, __builtin_amdgcn_perm(lt.t0, c ^ b, sel_byte(0))) ^ (c >> 8);
}

// shift(c, D) through operator `op` (4 x 256 entries, one LDS copy).
__device__ __forceinline__ uint32_t shift_op(const char* lds, uint32_t op, uint32_t c) {
  const uint32_t base = PDB_MAIN_BYTES + op * 4096u;
  const uint32_t v0 = lds_u32(lds, base + ((c & 0xffu) << 2));
  const uint32_t v1 = lds_u32(lds, base + 1024u + (((c >> 8) & 0xffu) << 2));
  const uint32_t v2 = lds_u32(lds, base + 2048u + (((c >> 16) & 0xffu) << 2));
  const uint32_t v3 = lds_u32(lds, base + 3072u + ((c >> 24) << 2));
  return (v0 ^ v1) ^ (v2 ^ v3);
}

// shift(c, D_op) ^ y
__device__ __forceinline__ uint32_t shift_op_x(const char* lds, uint32_t op, uint32_t c, uint32_t y) {
  const uint32_t base = PDB_MAIN_BYTES + op * 4096u;
  const uint32_t v0 = lds_u32(lds, base + ((c & 0xffu) << 2));
  const uint32_t v1 = lds_u32(lds, base + 1024u + (((c >> 8) & 0xffu) << 2));
  const uint32_t v2 = lds_u32(lds, base + 2048u + (((c >> 16) & 0xffu) << 2));
  const uint32_t v3 = lds_u32(lds, base + 3072u + ((c >> 24) << 2));
  return xor3(xor3(v0, v1, v2), v3, y);
}

// Same fold with the partner values moved by DPP (levels 0-3, row_shl), ds_swizzle (level 4,
// xor 16 within 32-lane halves) and readlane (level 5): one LDS round trip fewer per level
// than ds_bpermute.  Result valid in lane 0.
template <bool kL5Twice = false>
__device__ __forceinline__ uint32_t wave_tree_dpp(const char* lds, uint32_t lane, uint32_t c) {
  uint32_t y;
  y = __builtin_amdgcn_update_dpp(0u, c, 0x101, 0xF, 0xF, false);  // row_shl:1
  if ((lane & 1u) == 0) c = shift_op_x(lds, 0, c, y);
  y = __builtin_amdgcn_update_dpp(0u, c, 0x102, 0xF, 0xF, false);  // row_shl:2
  if ((lane & 3u) == 0) c = shift_op_x(lds, 1, c, y);
  y = __builtin_amdgcn_update_dpp(0u, c, 0x104, 0xF, 0xF, false);  // row_shl:4
  if ((lane & 7u) == 0) c = shift_op_x(lds, 2, c, y);
  y = __builtin_amdgcn_update_dpp(0u, c, 0x108, 0xF, 0xF, false);  // row_shl:8
  if ((lane & 15u) == 0) c = shift_op_x(lds, 3, c, y);
  y = __builtin_amdgcn_ds_swizzle(c, 0x401F);  // bitmask mode: lane ^ 16 within 32
  if ((lane & 31u) == 0) c = shift_op_x(lds, 4, c, y);
  y = __builtin_amdgcn_readlane(c, 32);
  if (lane == 0) {
    if constexpr (kL5Twice)  // slot 5 left free (LDS scratch): shift 2P = shift P twice
      c = shift_op_x(lds, 4, shift_op(lds, 4, c), y);
    else
      c = shift_op_x(lds, 5, c, y);
  }
  return c;
}

__device__ __forceinline__ uint32_t finalize(uint32_t raw, uint32_t flags) {
  const uint32_t crc = ~raw;
  return (flags & PDB_CRC_MASK_OUTPUT) ? pdb_mask(crc) : crc;
}

// Unaligned 32-bit little-endian load that never touches an aligned dword holding no byte of
// [q, q+4).
__device__ __forceinline__ uint32_t ld32u(const uint8_t* q) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(q);
  const uint32_t s = static_cast<uint32_t>(a & 3u);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~static_cast<uintptr_t>(3));
  const uint32_t lo = w[0];
  if (s == 0) return lo;
  return __builtin_amdgcn_alignbyte(w[1], lo, s);
}

// Stage the table image into LDS: T0..T3 written 32x (8 x 16-B stores per entry); tree
// operators catalog[kTree .. kTree+5] -> slots 0..5; catalog[kHorner] -> slot 6 (if >= 0).
template <int kTree, int kHorner, int kSlot7 = -1, bool kSkipSlot5 = false>
__device__ __forceinline__ void stage_tables(char* lds, const uint32_t* __restrict__ tabs) {
  for (uint32_t i = threadIdx.x; i < 4u * 256u * 8u; i += blockDim.x) {
    const uint32_t k = i >> 11, b = (i >> 3) & 255u, part = i & 7u;
    const uint32_t v = tabs[k * 256u + b];
    const uint32_t addr = ((k >> 1) << 16) | (b << 8) | ((k & 1u) << 7) | (part << 4);
    *reinterpret_cast<u32x4*>(lds + addr) = u32x4{v, v, v, v};
  }
  const u32x4* cat = reinterpret_cast<const u32x4*>(tabs + 1024);
  constexpr uint32_t nslots = kSlot7 >= 0 ? 8u : (kHorner >= 0 ? 7u : 6u);
  for (uint32_t i = threadIdx.x; i < nslots * 256u; i += blockDim.x) {
    const uint32_t slot = i >> 8;
    if (kSkipSlot5 && slot == 5) continue;
    const uint32_t src = slot < 6 ? kTree + slot
                                  : (slot == 6 ? static_cast<uint32_t>(kHorner) : static_cast<uint32_t>(kSlot7));
    *reinterpret_cast<u32x4*>(lds + PDB_MAIN_BYTES + i * 16u) = cat[src * 256u + (i & 255u)];
  }
}

__device__ __forceinline__ uint64_t wave_id_uniform() {
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  return static_cast<uint64_t>(blockIdx.x) * kWavesPerWg + w;
}

// ---- fixed-stride batch, 4-KiB fast path ------------------------------------------------------
// len == 4096, base and stride 16-B aligned, one round, no head.  Lane l owns kNP pieces of
// P = 64/kNP contiguous bytes: piece p at p*(4096/kNP) + l*P.  kNP = 1 is the lane-contiguous
// layout (each 16-B load instruction spans 4 KiB); kNP = 4 makes every load instruction read
// 1 KiB contiguous (coalesced) at the price of a Horner shift over the (4096/kNP - P)-byte gap
// between a lane's pieces (LDS slot 6).  Each wave walks blocks b, b+W, ... (W = waves in the
// grid) with kDepth blocks of loads in flight ahead of the one it hashes.
template <int kNP>
__device__ __forceinline__ void load4k(u32x4 (&v)[4], const uint8_t* base, uint64_t stride, uint64_t b,
                                       uint32_t lane) {
  constexpr uint32_t P = 64u / kNP, gap = 4096u / kNP, per = 4u / kNP;
  const uint8_t* blk = base + b * stride + lane * P;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    v[i] = *reinterpret_cast<const u32x4*>(blk + (i / per) * gap + (i % per) * 16u);
}

// The lane's 16 dwords are hashed as NCH independent slice-by-4 chains (ILP: half or a quarter
// of the serial LDS round trips), then folded with the slot-6 operator "shift by the distance
// between consecutive chain ends" (32 B for kNP=1, 2048 B for kNP=2, 1024 B for kNP=4).
template <int kNP>
__device__ __forceinline__ uint32_t hash4k(const char* lds, const LaneTabs& lt, uint32_t lane,
                                           uint32_t c0, const u32x4 (&v)[4]) {
  const uint32_t d[16] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                          v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
  constexpr int NCH = kNP == 1 ? 2 : kNP;
  constexpr int per = 16 / NCH;
  uint32_t x[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) x[ch] = (ch == 0 ? c0 : 0u) ^ d[ch * per];
#pragma unroll
  for (int i = 1; i <= per; ++i)
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) x[ch] = step4x(lds, lt, x[ch], i < per ? d[ch * per + i] : 0u);
  uint32_t c = x[0];
#pragma unroll
  for (int ch = 1; ch < NCH; ++ch) c = shift_op_x(lds, PDB_SLOT_HORNER, c, x[ch]);
  return wave_tree_dpp(lds, lane, c);
}

template <int kNP, int kDepth, bool kIssueFirst = false>
__global__ __launch_bounds__(kThreads) void crc_fast4k_kernel(
    const uint32_t* __restrict__ tabs, const uint8_t* __restrict__ base, uint64_t stride,
    uint64_t nblk, uint32_t flags, uint32_t init, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerWg;
  const uint64_t b0 = wave_id_uniform();
  // Issue the first kDepth blocks' loads before staging the tables: the table copy then
  // overlaps the first HBM round trip.
  u32x4 buf[kDepth][4];
#pragma unroll
  for (int k = 0; k < kDepth; ++k) {
    const uint64_t b = b0 + k * nw;
    load4k<kNP>(buf[k], base, stride, b < nblk ? b : (nblk - 1), lane);
  }
  constexpr int kTree = kNP == 1 ? PDB_CAT_TREE64 : (kNP == 2 ? PDB_CAT_TREE32 : PDB_CAT_TREE16);
  constexpr int kHorner = kNP == 1 ? PDB_CAT_TREE32 : (kNP == 2 ? PDB_CAT_S2048 : PDB_CAT_S1024);
  stage_tables<kTree, kHorner>(lds, tabs);
  __syncthreads();
  const LaneTabs lt = lane_tabs(lane);
  const uint32_t init_raw = (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu;
  // Results are parked in a register (lane j holds the j-th block's CRC of the current 64-block
  // window) and flushed with one scattered 64-lane store per window: a per-block store from
  // lane 0 would sit in vmcnt behind the next block's loads and make every wait drain it.
  uint32_t res = 0;
  uint32_t it = 0;
  uint64_t win0 = b0;  // first block of the current window
  for (uint64_t b = b0; b < nblk; b += kDepth * nw) {
#pragma unroll
    for (int k = 0; k < kDepth; ++k) {
      const uint64_t bk = b + k * nw;
      if (bk >= nblk) break;  // wave-uniform
      u32x4 cur[4] = {buf[k][0], buf[k][1], buf[k][2], buf[k][3]};
      const uint64_t bn = bk + kDepth * nw;
      load4k<kNP>(buf[k], base, stride, bn < nblk ? bn : bk, lane);  // clamp: valid block
      if constexpr (kIssueFirst) __builtin_amdgcn_sched_barrier(0);
      const uint32_t c = hash4k<kNP>(lds, lt, lane, lane == 0 ? init_raw : 0u, cur);
      const uint32_t v = finalize(__builtin_amdgcn_readfirstlane(c), flags);
      if (lane == (it & 63u)) res = v;
      if ((++it & 63u) == 0) {
        out[win0 + static_cast<uint64_t>(lane) * nw] = res;
        win0 += 64 * nw;
      }
    }
  }
  if ((it & 63u) && lane < (it & 63u)) out[win0 + static_cast<uint64_t>(lane) * nw] = res;
}

// ---- fixed-stride batch, 4-KiB ping-pong path ----------------------------------------------------
// crc_fast4k_kernel<2,1> with two named load buffers and a scheduling barrier right after each
// load issue, so the next block's 4 KiB is in flight for the WHOLE hash of the current block
// (hipcc otherwise sinks the loads a third of the way into the chain to reuse registers).
__global__ __launch_bounds__(kThreads) void crc_pingpong4k_kernel(
    const uint32_t* __restrict__ tabs, const uint8_t* __restrict__ base, uint64_t stride,
    uint64_t nblk, uint32_t flags, uint32_t init, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerWg;
  const uint64_t b0 = wave_id_uniform();
  u32x4 A[4], B[4];
  load4k<2>(A, base, stride, b0 < nblk ? b0 : nblk - 1, lane);
  stage_tables<PDB_CAT_TREE32, PDB_CAT_S2048>(lds, tabs);
  __syncthreads();
  if (b0 >= nblk) return;
  const LaneTabs lt = lane_tabs(lane);
  const uint32_t init_raw = (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu;
  const uint32_t c0 = lane == 0 ? init_raw : 0u;
  uint32_t res = 0, it = 0;
  uint64_t win0 = b0;
  auto emit = [&](uint32_t c) {
    const uint32_t v = finalize(__builtin_amdgcn_readfirstlane(c), flags);
    if (lane == (it & 63u)) res = v;
    if ((++it & 63u) == 0) {
      out[win0 + static_cast<uint64_t>(lane) * nw] = res;
      win0 += 64 * nw;
    }
  };
  for (uint64_t b = b0; b < nblk; b += 2 * nw) {
    const uint64_t b1 = b + nw, b2 = b + 2 * nw;
    load4k<2>(B, base, stride, b1 < nblk ? b1 : b, lane);
    __builtin_amdgcn_sched_barrier(0);
    emit(hash4k<2>(lds, lt, lane, c0, A));
    if (b1 >= nblk) break;
    load4k<2>(A, base, stride, b2 < nblk ? b2 : b1, lane);
    __builtin_amdgcn_sched_barrier(0);
    emit(hash4k<2>(lds, lt, lane, c0, B));
  }
  if ((it & 63u) && lane < (it & 63u)) out[win0 + static_cast<uint64_t>(lane) * nw] = res;
}

// ---- fixed-stride batch, 4-KiB packed-tree path ------------------------------------------------
// Same per-block loads and chains as crc_fast4k_kernel<2,1> (64 lanes per block, two 32-B pieces
// per lane), but a wave hashes 4 blocks back to back and folds their 4 x 64 lane partials in ONE
// packed tree: level 0 pairs lanes (2m, 2m+1) of blocks {0,1} and then {2,3} with every lane
// doing useful work, level 1 pairs quads of all 4 blocks in one full-wave round, levels 2-5 run
// once for all 4 blocks.  7 shift operations per 4 blocks instead of 24.
__device__ __forceinline__ uint32_t sel(bool c, uint32_t a, uint32_t b) { return c ? a : b; }

// Returns block (lane & 3)'s raw state in lanes 0..3.
__device__ __forceinline__ uint32_t tree4_packed(const char* lds, uint32_t u, uint32_t p0, uint32_t p1,
                                                 uint32_t p2, uint32_t p3) {
  const bool odd = u & 1u;
  // level 0 (shift 32): even lane 2m -> block 0/2 pair m, odd lane 2m+1 -> block 1/3 pair m
  const uint32_t p0n = __builtin_amdgcn_update_dpp(0u, p0, 0x101, 0xF, 0xF, false);  // p0[L+1]
  const uint32_t p1p = __builtin_amdgcn_update_dpp(0u, p1, 0x111, 0xF, 0xF, false);  // p1[L-1]
  const uint32_t r0 = shift_op_x(lds, 0, sel(odd, p1p, p0), sel(odd, p1, p0n));
  const uint32_t p2n = __builtin_amdgcn_update_dpp(0u, p2, 0x101, 0xF, 0xF, false);
  const uint32_t p3p = __builtin_amdgcn_update_dpp(0u, p3, 0x111, 0xF, 0xF, false);
  const uint32_t r1 = shift_op_x(lds, 0, sel(odd, p3p, p2), sel(odd, p3, p2n));
  // level 1 (shift 64): lane 4j+r -> block r pair j.  r<2 reads r0 at L, L+2; r>=2 reads r1 at L-2, L
  const bool hi = u & 2u;
  const uint32_t r0n = __builtin_amdgcn_update_dpp(0u, r0, 0x102, 0xF, 0xF, false);  // r0[L+2]
  const uint32_t r1p = __builtin_amdgcn_update_dpp(0u, r1, 0x112, 0xF, 0xF, false);  // r1[L-2]
  uint32_t v = shift_op_x(lds, 1, sel(hi, r1p, r0), sel(hi, r1, r0n));
  // levels 2..5: lane 4j+r holds block r; pair (L, L + 4*2^(k-2))
  uint32_t y = __builtin_amdgcn_update_dpp(0u, v, 0x104, 0xF, 0xF, false);  // row_shl:4
  if ((u & 4u) == 0) v = shift_op_x(lds, 2, v, y);
  y = __builtin_amdgcn_update_dpp(0u, v, 0x108, 0xF, 0xF, false);  // row_shl:8
  if ((u & 12u) == 0) v = shift_op_x(lds, 3, v, y);
  y = __builtin_amdgcn_ds_swizzle(v, 0x401F);  // lane ^ 16
  if ((u & 28u) == 0) v = shift_op_x(lds, 4, v, y);
  y = __shfl_down(v, 32, 64);
  if ((u & 60u) == 0) v = shift_op_x(lds, 5, v, y);
  return v;
}

__device__ __forceinline__ uint32_t partial4k(const char* lds, const LaneTabs& lt, uint32_t c0,
                                              const u32x4 (&v)[4]) {
  uint32_t xa = c0 ^ v[0].x, xb = v[2].x;
  const uint32_t da[8] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
  const uint32_t db[8] = {v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
#pragma unroll
  for (int i = 1; i <= 8; ++i) {
    xa = step4x(lds, lt, xa, i < 8 ? da[i] : 0u);
    xb = step4x(lds, lt, xb, i < 8 ? db[i] : 0u);
  }
  return shift_op_x(lds, PDB_SLOT_HORNER, xa, xb);  // shift 2048
}

template <int kSync>
__global__ __launch_bounds__(kThreads) void crc_pack4k_kernel(
    const uint32_t* __restrict__ tabs, const uint8_t* __restrict__ base, uint64_t stride,
    uint64_t nblk, uint32_t flags, uint32_t init, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  const uint32_t u = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerWg;
  const uint64_t w = wave_id_uniform();
  u32x4 buf[4];
  load4k<2>(buf, base, stride, w < nblk ? w : nblk - 1, u);
  stage_tables<PDB_CAT_TREE32, PDB_CAT_S2048>(lds, tabs);
  __syncthreads();
  if (kSync == 0 && w >= nblk) return;
  const LaneTabs lt = lane_tabs(u);
  const uint32_t init_raw = (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu;
  const uint32_t c0 = u == 0 ? init_raw : 0u;
  uint32_t res = 0, it = 0;
  // kSync: the workgroup's 16 waves (16 consecutive blocks) stay in lock step, one barrier per
  // 4-block group, so their outstanding loads cover one compact 64-KiB span at a time.
  const uint64_t wg_first = static_cast<uint64_t>(blockIdx.x) * kWavesPerWg;
  if (kSync > 0 && wg_first >= nblk) return;
  uint32_t grp = 0;
  uint64_t win0 = w;
  for (uint64_t g = w, gw = wg_first; (kSync > 0 ? gw : g) < nblk; g += 4 * nw, gw += 4 * nw) {
    if constexpr (kSync > 0) {
      if ((grp++ % kSync) == 0) __syncthreads();
    }
    uint32_t p[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint64_t bk = g + r * nw;
      u32x4 cur[4] = {buf[0], buf[1], buf[2], buf[3]};
      const uint64_t bn = bk + nw;
      if (bn < nblk) load4k<2>(buf, base, stride, bn, u);  // wave-uniform
      p[r] = bk < nblk ? partial4k(lds, lt, c0, cur) : 0u;
    }
    const uint32_t v = tree4_packed(lds, u, p[0], p[1], p[2], p[3]);
    // lane 4j+r of the 64-block window holds block (window + (4j+r)*nw): move lanes 0..3's
    // results up by 4*(group mod 16) with one DPP-free bpermute, park, flush every 16 groups.
    const uint32_t slot = (it & 15u) * 4u;
    const uint32_t vv = __shfl(v, u & 3u, 64);
    if ((u & ~3u) == slot) res = finalize(vv, flags);
    if ((++it & 15u) == 0) {
      const uint64_t bo = win0 + static_cast<uint64_t>(u) * nw;
      if (bo < nblk) out[bo] = res;
      win0 += 64 * nw;
    }
  }
  if (it & 15u) {
    const uint64_t bo = win0 + static_cast<uint64_t>(u) * nw;
    if (u < (it & 15u) * 4u && bo < nblk) out[bo] = res;
  }
}

// Dynamic variant of the packed kernel: workgroup g owns blocks [g*N/G, (g+1)*N/G); each wave
// takes 4 consecutive blocks at a time from an LDS counter (operator slot 7 is unused here) and
// writes their 4 CRCs with one 16-B store.
__global__ __launch_bounds__(kThreads) void crc_pack4k_dyn_kernel(
    const uint32_t* __restrict__ tabs, const uint8_t* __restrict__ base, uint64_t stride,
    uint64_t nblk, uint32_t flags, uint32_t init, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  uint32_t* ctr = reinterpret_cast<uint32_t*>(lds + PDB_MAIN_BYTES + 7 * 4096u);
  const uint32_t u = threadIdx.x & 63u;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t g_lo = nblk * blockIdx.x / gridDim.x, g_hi = nblk * (blockIdx.x + 1) / gridDim.x;
  uint64_t grp = g_lo + 4u * wid;  // first group of this wave (static), then from the counter
  u32x4 buf[4];
  load4k<2>(buf, base, stride, grp < g_hi ? grp : (nblk ? nblk - 1 : 0), u);
  stage_tables<PDB_CAT_TREE32, PDB_CAT_S2048>(lds, tabs);
  if (threadIdx.x == 0) *ctr = kWavesPerWg;  // next group, in groups relative to g_lo
  __syncthreads();
  const LaneTabs lt = lane_tabs(u);
  const uint32_t init_raw = (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu;
  const uint32_t c0 = u == 0 ? init_raw : 0u;
  while (grp < g_hi) {
    uint32_t r0 = 0;
    if (u == 0) r0 = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint64_t ngrp = g_lo + 4u * static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(r0));
    uint32_t p[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint64_t bk = grp + r;
      u32x4 cur[4] = {buf[0], buf[1], buf[2], buf[3]};
      const uint64_t bn = r < 3 ? bk + 1 : ngrp;
      if (bn < g_hi) load4k<2>(buf, base, stride, bn, u);  // wave-uniform
      p[r] = bk < g_hi ? partial4k(lds, lt, c0, cur) : 0u;
    }
    const uint32_t v = tree4_packed(lds, u, p[0], p[1], p[2], p[3]);
    if (u < 4 && grp + u < g_hi) out[grp + u] = finalize(v, flags);
    grp = ngrp;
  }
}

// ---- fixed-stride batch, 4-KiB team path ----------------------------------------------------
// A wave hashes T = 64/kG consecutive 4-KiB blocks at once: team t (lanes [t*kG, (t+1)*kG))
// owns block t.  Within a team, lane u owns R = 4096/(32*kG) pieces of 32 B, piece r at
// r*32*kG + 32*u, so every 16-B load instruction covers T blocks x kG lanes at a 32-B lane
// stride.  Each piece is an independent 8-step chain; the R chains fold with "shift by
// 32*kG bytes" (slot 6), then a log2(kG)-level team tree (slots 0.., shift by 32 << k) whose
// VALU/LDS instructions serve all T blocks at once -- the per-block tree cost drops by T.
template <int kG>
__device__ __forceinline__ uint32_t team_tree(const char* lds, uint32_t u, uint32_t c) {
  uint32_t y;
  y = __builtin_amdgcn_update_dpp(0u, c, 0x101, 0xF, 0xF, false);
  if ((u & 1u) == 0) c = shift_op_x(lds, 0, c, y);
  y = __builtin_amdgcn_update_dpp(0u, c, 0x102, 0xF, 0xF, false);
  if ((u & 3u) == 0) c = shift_op_x(lds, 1, c, y);
  y = __builtin_amdgcn_update_dpp(0u, c, 0x104, 0xF, 0xF, false);
  if ((u & 7u) == 0) c = shift_op_x(lds, 2, c, y);
  y = __builtin_amdgcn_update_dpp(0u, c, 0x108, 0xF, 0xF, false);
  if ((u & 15u) == 0) c = shift_op_x(lds, 3, c, y);
  if constexpr (kG >= 32) {
    y = __builtin_amdgcn_ds_swizzle(c, 0x401F);
    if ((u & 31u) == 0) c = shift_op_x(lds, 4, c, y);
  }
  if constexpr (kG >= 64) {
    y = __builtin_amdgcn_readlane(c, 32);
    if (u == 0) c = shift_op_x(lds, 5, c, y);
  }
  return c;
}

template <int kG, int kDepth>
__global__ __launch_bounds__(kThreads) void crc_team4k_kernel(
    const uint32_t* __restrict__ tabs, const uint8_t* __restrict__ base, uint64_t stride,
    uint64_t nblk, uint32_t flags, uint32_t init, uint32_t* __restrict__ out) {
  constexpr uint32_t T = 64 / kG;             // blocks per wave-iteration
  constexpr uint32_t R = 4096 / (32 * kG);    // 32-B pieces per lane per block
  constexpr uint32_t ROW = 32 * kG;           // bytes between a lane's pieces
  constexpr int kFold = kG == 32 ? PDB_CAT_S1024 : (kG == 16 ? 5 /* 512 */ : PDB_CAT_S2048);
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t t = lane / kG, u = lane % kG;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerWg;
  const uint64_t ngroups = (nblk + T - 1) / T;  // wave-iterations needed in total
  const uint64_t g0 = wave_id_uniform();

  auto load = [&](u32x4 (&v)[2 * R], uint64_t g) {
    uint64_t b = g * T + t;
    if (b >= nblk) b = nblk - 1;  // clamp: a valid block (result discarded)
    const uint8_t* p = base + b * stride + u * 32u;
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      v[2 * r] = *reinterpret_cast<const u32x4*>(p + r * ROW);
      v[2 * r + 1] = *reinterpret_cast<const u32x4*>(p + r * ROW + 16u);
    }
  };

  u32x4 nxt[2 * R];
  if constexpr (kDepth > 0) load(nxt, g0 < ngroups ? g0 : 0);
  stage_tables<PDB_CAT_TREE32, kFold>(lds, tabs);
  __syncthreads();
  const LaneTabs lt = lane_tabs(lane);
  const uint32_t init_raw = (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu;
  for (uint64_t g = g0; g < ngroups; g += nw) {
    u32x4 cur[2 * R];
    if constexpr (kDepth > 0) {
#pragma unroll
      for (uint32_t i = 0; i < 2 * R; ++i) cur[i] = nxt[i];
      const uint64_t gn = g + nw;
      load(nxt, gn < ngroups ? gn : g);
    } else {
      load(cur, g);
    }
    uint32_t x[R];
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) x[r] = cur[2 * r].x ^ ((r == 0 && u == 0) ? init_raw : 0u);
#pragma unroll
    for (int i = 1; i <= 8; ++i) {
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) {
        const u32x4& a = cur[2 * r];
        const u32x4& bq = cur[2 * r + 1];
        const uint32_t w = i == 1 ? a.y : i == 2 ? a.z : i == 3 ? a.w : i == 4 ? bq.x
                         : i == 5 ? bq.y : i == 6 ? bq.z : i == 7 ? bq.w : 0u;
        x[r] = step4x(lds, lt, x[r], w);
      }
    }
    uint32_t c = x[0];
#pragma unroll
    for (uint32_t r = 1; r < R; ++r) c = shift_op_x(lds, PDB_SLOT_HORNER, c, x[r]);
    c = team_tree<kG>(lds, u, c);
    const uint64_t b = g * T + t;
    if (u == 0 && b < nblk) out[b] = finalize(c, flags);
  }
}

// ---- generic stream kernel: any length, any alignment, fixed-stride / descriptors / sstable --
// One wave per block; the wave walks its blocks (i, i+W, ...) and each block's rounds as one
// software-pipelined stream of items: while item (i, r) is hashed, item (i, r+1) -- or round 0
// of the next block, with its descriptor and head words -- is already loading.
//   block of n bytes = head (t = n % 32 bytes) + K = n / 32 pieces of 32 B at p + t + 32c;
//   piece c -> lane c % 64, j = c / 64; a round is 4 KiB: lane u hashes pieces j = 2r (at
//   4096r + 32u) and 2r+1 (2048 higher) as two independent chains, folded with "shift 2048"
//   (slot 7); rounds chain per lane with "shift 2016" (slot 6) -- the 4-KiB fast path's
//   geometry generalised.  The head is hashed by every lane (broadcast words) from the Extend
//   seed and becomes lane 0's starting state; lanes are rotated when K % 64 != 0 so lane v's
//   partial ends 32*(63-v) bytes before the end; then the 6-level DPP tree (slots 0..5: 32 << k).
struct BlkDesc {
  const uint8_t* p;
  uint32_t n;
  uint32_t init_raw;  // ~Extend seed
};

struct FixedSrc {
  const uint8_t* base;
  uint64_t stride;
  uint32_t len;
  uint32_t init_raw;
  __device__ __forceinline__ BlkDesc get(uint64_t i) const { return {base + i * stride, len, init_raw}; }
};

struct DescSrc {
  const uint8_t* base;
  const pdb_blk* blk;
  uint32_t flags;
  __device__ __forceinline__ BlkDesc get(uint64_t i) const {
    const pdb_blk d = blk[i];
    return {base + d.off, d.len, (flags & PDB_CRC_USE_INIT) ? ~d.init : 0xFFFFFFFFu};
  }
};

// sstable handle: CRC over contents || type (table/table_builder.cc:197-198; format.cc:98).
struct SstSrc {
  uint8_t* buf;
  const pdb_block_handle* h;
  __device__ __forceinline__ BlkDesc get(uint64_t i) const {
    const pdb_block_handle x = h[i];
    return {buf + x.offset, static_cast<uint32_t>(x.size + 1), 0xFFFFFFFFu};
  }
};

struct OutSink {
  uint32_t* out;
  uint32_t flags;
  __device__ __forceinline__ void put(uint64_t i, uint32_t raw, const BlkDesc&) const {
    out[i] = finalize(raw, flags);
  }
};

struct VerifySink {
  const uint32_t* expected;
  uint8_t* ok;
  uint32_t* nbad;
  uint32_t flags;
  __device__ __forceinline__ void put(uint64_t i, uint32_t raw, const BlkDesc&) const {
    const bool good = finalize(raw, flags) == expected[i];
    if (ok) ok[i] = good ? 1 : 0;
    if (!good && nbad) atomicAdd(nbad, 1u);
  }
};

// Seal: EncodeFixed32(trailer + 1, Mask(crc)) at contents + size + 1 = p + n.
struct SealSink {
  __device__ __forceinline__ void put(uint64_t, uint32_t raw, const BlkDesc& d) const {
    uint8_t* tr = const_cast<uint8_t*>(d.p) + d.n;
    const uint32_t m = pdb_mask(~raw);
    tr[0] = static_cast<uint8_t>(m);
    tr[1] = static_cast<uint8_t>(m >> 8);
    tr[2] = static_cast<uint8_t>(m >> 16);
    tr[3] = static_cast<uint8_t>(m >> 24);
  }
};

// ReadBlock's check: Unmask(DecodeFixed32(data + n + 1)) == crc (format.cc:96-104).
struct SstVerifySink {
  uint8_t* ok;
  uint32_t* nbad;
  __device__ __forceinline__ void put(uint64_t i, uint32_t raw, const BlkDesc& d) const {
    const uint8_t* tr = d.p + d.n;
    const uint32_t stored = static_cast<uint32_t>(tr[0]) | (static_cast<uint32_t>(tr[1]) << 8) |
                            (static_cast<uint32_t>(tr[2]) << 16) | (static_cast<uint32_t>(tr[3]) << 24);
    const bool good = pdb_unmask(stored) == ~raw;
    if (ok) ok[i] = good ? 1 : 0;
    if (!good && nbad) atomicAdd(nbad, 1u);
  }
};

// Raw (possibly misaligned) 32-B piece: e[0..8] are the aligned dwords covering [q - s, q - s + 36).
struct RawPiece {
  uint32_t e[9];
};

__device__ __forceinline__ void issue_piece(RawPiece& r, const uint8_t* q, uint32_t s) {
  const u32x4a4* v = reinterpret_cast<const u32x4a4*>(q - s);
  const u32x4a4 x0 = v[0], x1 = v[1];
  r.e[0] = x0.x; r.e[1] = x0.y; r.e[2] = x0.z; r.e[3] = x0.w;
  r.e[4] = x1.x; r.e[5] = x1.y; r.e[6] = x1.z; r.e[7] = x1.w;
  // the 9th dword holds the piece's last byte(s) only when misaligned (never past the block)
  r.e[8] = s ? *reinterpret_cast<const uint32_t*>(q - s + 32) : 0u;
}

// Chain over one 32-B piece: returns shift(x0_state ^ piece ...), i.e. the raw state after the
// piece starting from `start` (injected into the first word).
__device__ __forceinline__ uint32_t chain_piece(const char* lds, const LaneTabs& lt, uint32_t start,
                                                const RawPiece& r, uint32_t s) {
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = s ? __builtin_amdgcn_alignbyte(r.e[j + 1], r.e[j], s) : r.e[j];
  uint32_t x = start ^ w[0];
#pragma unroll
  for (int j = 1; j <= 8; ++j) x = step4x(lds, lt, x, j < 8 ? w[j] : 0u);
  return x;
}

// kSync (equal-length sources): the workgroup's 16 waves advance one item at a time in lock
// step (one barrier per item), so their outstanding loads stay within one compact span of
// consecutive blocks -- DRAM row locality that free-running waves lose as they drift apart
// (measured on the 4-KiB path: +8 %).
// kDyn (unequal lengths: descriptors, sstable handles): workgroup g owns the contiguous block
// range [g*N/G, (g+1)*N/G) and its 16 waves take the next block from an LDS counter (LDS slot 5,
// freed by folding tree level 5 as two "shift 512"s): the CU's work is balanced and its
// outstanding loads stay on a compact run of consecutive blocks.
template <class Src, class Sink, int kSync, bool kDyn = false>
__global__ __launch_bounds__(kThreads) void crc_stream_kernel(const uint32_t* __restrict__ tabs,
                                                               Src src, uint64_t nblk, Sink sink) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  stage_tables<PDB_CAT_TREE32, PDB_CAT_H2016, PDB_CAT_S2048, kDyn>(lds, tabs);
  uint32_t* ctr = reinterpret_cast<uint32_t*>(lds + PDB_MAIN_BYTES + 5 * 4096u);
  const uint64_t g_lo = nblk * blockIdx.x / gridDim.x, g_hi = nblk * (blockIdx.x + 1) / gridDim.x;
  if (kDyn && threadIdx.x == 0) *ctr = kWavesPerWg;  // next block, relative to g_lo
  __syncthreads();
  const uint32_t u = threadIdx.x & 63u;
  const LaneTabs lt = lane_tabs(u);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerWg;
  auto next_block = [&](uint64_t cur) -> uint64_t {
    if constexpr (kDyn) {
      uint32_t r = 0;
      if (u == 0) r = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return g_lo + __builtin_amdgcn_readfirstlane(r);
    } else {
      return cur + nw;
    }
  };
  const uint64_t nend = kDyn ? g_hi : nblk;
  uint64_t i = kDyn ? g_lo + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : wave_id_uniform();
  bool active = i < nend;
  if (kSync == 0 && !active) return;

  // the item being loaded: block d, round k
  BlkDesc d{};
  uint32_t k = 0;
  RawPiece na, nb;
  uint32_t nhw = 0, nhb = 0;
  auto issue = [&](const BlkDesc& bd, uint32_t kk) {
    const uint32_t t = bd.n & 31u, K = bd.n >> 5;
    const uint8_t* q0 = bd.p + t;
    const uint32_t s = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(q0) & 3u);
    const uint32_t ca = u + (kk << 7), cb = ca + 64u;
    if (ca < K) issue_piece(na, q0 + static_cast<uint64_t>(ca) * 32u, s);
    if (cb < K) issue_piece(nb, q0 + static_cast<uint64_t>(cb) * 32u, s);
    if (kk == 0) {
      const uint32_t lead = t & 3u, nh = t >> 2;
      if (u >= 1 && u <= nh) nhw = ld32u(bd.p + lead + 4u * (u - 1));
      if (u == 0 && lead) {
        uint32_t v = bd.p[0];
        if (lead > 1) v |= static_cast<uint32_t>(bd.p[1]) << 8;
        if (lead > 2) v |= static_cast<uint32_t>(bd.p[2]) << 16;
        nhb = v;
      }
    }
  };
  if (active) {
    d = src.get(i);
    issue(d, 0);
  }
  uint32_t acc = 0;
  // kSync (equal lengths): every wave of the workgroup runs as many items as its first wave
  // (the one with the most blocks), so a plain barrier per item needs no LDS reduction.
  uint64_t items_left = 0, item = 0;
  if constexpr (kSync > 0) {
    const uint64_t wg_first = static_cast<uint64_t>(blockIdx.x) * kWavesPerWg;
    if (wg_first >= nblk) return;
    const uint32_t n0 = src.get(wg_first).n, K0 = n0 >> 5;
    items_left = ((nblk - wg_first + nw - 1) / nw) * (K0 ? (K0 + 127u) >> 7 : 1u);
  }
  for (;;) {
    if constexpr (kSync > 0) {
      if (items_left-- == 0) break;
      if ((item++ % kSync) == 0) __syncthreads();
      if (!active) continue;
    }
    const RawPiece ca_ = na, cb_ = nb;
    const uint32_t chw = nhw, chb = nhb;
    const BlkDesc cd = d;
    const uint32_t ck = k;
    const uint32_t K = cd.n >> 5;
    const uint32_t R = K ? (K + 127u) >> 7 : 1u;
    const bool last_round = ck + 1 >= R;
    const uint64_t ni = last_round ? next_block(i) : i;
    const bool have_next = ni < nend;
    if (last_round && have_next) d = src.get(ni);
    k = last_round ? 0 : ck + 1;
    if (have_next) issue(d, k);

    if (ck == 0) {  // head: every lane hashes the same (broadcast) head bytes from the seed
      const uint32_t t = cd.n & 31u, lead = t & 3u, nh = t >> 2;
      uint32_t h = cd.init_raw;
      const uint32_t lb = __builtin_amdgcn_readfirstlane(chb);
      for (uint32_t j = 0; j < lead; ++j) h = step1(lds, lt, h, (lb >> (8 * j)) & 0xffu);
      for (uint32_t j = 0; j < nh; ++j) h = step4(lds, lt, h, __builtin_amdgcn_readlane(chw, j + 1));
      acc = (u == 0) ? h : 0u;
    }
    const uint32_t s = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(cd.p + (cd.n & 31u)) & 3u);
    const uint32_t ca = u + (ck << 7), cb = ca + 64u;
    if (cb < K) {
      const uint32_t start = ck ? shift_op(lds, PDB_SLOT_HORNER, acc) : acc;
      const uint32_t xa = chain_piece(lds, lt, start, ca_, s);
      const uint32_t xb = chain_piece(lds, lt, 0u, cb_, s);
      acc = shift_op_x(lds, 7, xa, xb);
    } else if (ca < K) {
      const uint32_t start = ck ? shift_op(lds, PDB_SLOT_HORNER, acc) : acc;
      acc = chain_piece(lds, lt, start, ca_, s);
    }
    if (last_round) {
      uint32_t raw = acc;
      if (K) {
        const uint32_t q = K & 63u;
        if (q) acc = __shfl(acc, (u + q) & 63u, 64);
        raw = wave_tree_dpp<kDyn>(lds, u, acc);
      }
      if (u == 0) sink.put(i, raw, cd);
      i = ni;
      if (!have_next) {
        active = false;
        if constexpr (kSync == 0) break;
      }
    }
  }
}

// ---- diagnostics ------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void read_stream_kernel(const u32x4* __restrict__ src,
                                                          uint64_t n16, uint32_t* __restrict__ out) {
  u32x4 acc = {0, 0, 0, 0};
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    acc ^= a ^ b ^ c ^ d;
  }
  for (; i < n16; i += stride) acc ^= src[i];
  uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
  for (int k = 32; k; k >>= 1) r ^= __shfl_xor(r, k, 64);
  if ((threadIdx.x & 63) == 0) atomicXor(out, r);
}

// Load-pattern calibration for 4-KiB blocks, no CRC work.
//   kPat 0: lane l reads bytes [64l, 64l+64) of the block (the fast path's pattern)
//   kPat 1: lane l reads 16 B at 16l + 1024j, j = 0..3 (each instruction 1 KiB contiguous)
//   kDepth: blocks in flight per wave; kAssign 0: wave-interleaved blocks, 1: contiguous per WG
template <int kPat, int kDepth, int kAssign, bool kSync = false>
__global__ __launch_bounds__(kThreads) void read_pattern4k_kernel(const uint8_t* __restrict__ base,
                                                                  uint64_t nblk,
                                                                  uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerWg;
  uint32_t acc = 0;
  uint64_t first, step, last;
  if constexpr (kAssign == 0) {
    first = wave_id_uniform();
    step = nw;
    last = nblk;
  } else {
    const uint64_t per = (nblk + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = blockIdx.x * per;
    first = lo + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    step = kWavesPerWg;
    last = lo + per < nblk ? lo + per : nblk;
  }
  const uint64_t wg_first = static_cast<uint64_t>(blockIdx.x) * kWavesPerWg;
  for (uint64_t b = first, bw = wg_first; (kSync ? bw : b) < last; b += step * kDepth, bw += step * kDepth) {
    if constexpr (kSync) __syncthreads();
    u32x4 x = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < kDepth; ++k) {
      const uint64_t bk = b + k * step;
      if (bk < last) {
        const uint8_t* blk = base + bk * 4096u;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t off = kPat == 0 ? lane * 64u + j * 16u
                             : (kPat == 1 ? lane * 16u + j * 1024u
                                          : lane * 32u + (j >> 1) * 2048u + (j & 1) * 16u);
          x ^= *reinterpret_cast<const u32x4*>(blk + off);
        }
      }
    }
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  for (int k = 32; k; k >>= 1) acc ^= __shfl_xor(acc, k, 64);
  if (lane == 0) atomicXor(out, acc);
}

__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Thread t writes dst[8t .. 8t+8) (bytes of the splitmix stream at byte_offset + 8t + j).
__global__ __launch_bounds__(256) void fill_splitmix_kernel(uint8_t* __restrict__ dst,
                                                            uint64_t nbytes, uint64_t seed,
                                                            uint64_t byte_offset) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint32_t sh = static_cast<uint32_t>(byte_offset & 7u);
  for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t * 8 < nbytes;
       t += stride) {
    const uint64_t g = byte_offset + t * 8;  // first global byte of this thread
    const uint64_t w0 = splitmix64_at(seed, g >> 3);
    uint64_t v = w0;
    if (sh) {
      const uint64_t w1 = splitmix64_at(seed, (g >> 3) + 1);
      v = (w0 >> (8 * sh)) | (w1 << (64 - 8 * sh));
    }
    if (t * 8 + 8 <= nbytes && (reinterpret_cast<uintptr_t>(dst) & 7u) == 0) {
      *reinterpret_cast<uint64_t*>(dst + t * 8) = v;
    } else {
      for (uint32_t j = 0; j < 8 && t * 8 + j < nbytes; ++j)
        dst[t * 8 + j] = static_cast<uint8_t>(v >> (8 * j));
    }
  }
}

uint32_t grid_for(const LaunchGeom& g, uint64_t nblk) {
  const uint64_t want = (nblk + kWavesPerWg - 1) / kWavesPerWg;
  return static_cast<uint32_t>(want < g.grid ? (want ? want : 1) : g.grid);
}

}  // namespace

int g_fast_variant = 0;  // diagnostics: pdb_diag_set_variant()

hipError_t launch_fixed(const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                        uint64_t stride, uint32_t len, uint64_t nblk, uint32_t flags, uint32_t init,
                        uint32_t* out, hipStream_t s) {
  if (nblk == 0) return hipSuccess;
  const dim3 grid(grid_for(g, nblk)), block(kThreads);
  const bool fast = len == 4096u && (reinterpret_cast<uintptr_t>(base) & 15u) == 0 &&
                    (stride & 15u) == 0;
  if (!fast) {
    const FixedSrc src{base, stride, len, (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu};
#define PDB_STREAM_FIXED(P)                                                                  \
  hipLaunchKernelGGL((crc_stream_kernel<FixedSrc, OutSink, P>), grid, block, 0, s, d_tables, src, nblk, \
                     OutSink{out, flags})
    switch (g_fast_variant) {  // A/B: lock-step period in items (0 = free-running)
      case 8: PDB_STREAM_FIXED(0); break;
      case 9: PDB_STREAM_FIXED(1); break;
      case 10: PDB_STREAM_FIXED(4); break;
      case 11: PDB_STREAM_FIXED(8); break;
      default:  // workgroup-local dynamic blocks: measured best (sstable layout +4 % over lock-step)
        hipLaunchKernelGGL((crc_stream_kernel<FixedSrc, OutSink, 0, true>), grid, block, 0, s, d_tables, src,
                           nblk, OutSink{out, flags});
        break;
    }
#undef PDB_STREAM_FIXED
    return hipGetLastError();
  }
#define PDB_FAST(NP, D)                                                                      \
  hipLaunchKernelGGL((crc_fast4k_kernel<NP, D>), grid, block, 0, s, d_tables, base, stride, nblk, \
                     flags, init, out)
#define PDB_TEAM(G, D)                                                                       \
  hipLaunchKernelGGL((crc_team4k_kernel<G, D>), grid, block, 0, s, d_tables, base, stride, nblk, \
                     flags, init, out)
  switch (g_fast_variant) {
    // A/B variants (tools/ab_fast.py); 0 = shipped default, measured best or tied on every box
    case 1: PDB_FAST(2, 1); break;  // 64-lane tree per block
    case 2: PDB_FAST(1, 1); break;  // 64-B lane pieces
    case 3: PDB_FAST(4, 1); break;  // coalesced 16-B pieces, 4 chains
    case 4: PDB_TEAM(32, 1); break;
    case 5: PDB_TEAM(16, 0); break;
    case 6: hipLaunchKernelGGL(crc_pingpong4k_kernel, grid, block, 0, s, d_tables, base, stride, nblk, flags, init, out); break;
    case 7: hipLaunchKernelGGL((crc_fast4k_kernel<2, 1, true>), grid, block, 0, s, d_tables, base, stride, nblk, flags, init, out); break;
    case 8: hipLaunchKernelGGL(crc_pack4k_kernel<0>, grid, block, 0, s, d_tables, base, stride, nblk, flags, init, out); break;
    case 9: hipLaunchKernelGGL(crc_pack4k_kernel<2>, grid, block, 0, s, d_tables, base, stride, nblk, flags, init, out); break;
    case 11: hipLaunchKernelGGL(crc_pack4k_dyn_kernel, grid, block, 0, s, d_tables, base, stride, nblk, flags, init, out); break;
    case 10: hipLaunchKernelGGL(crc_pack4k_kernel<4>, grid, block, 0, s, d_tables, base, stride, nblk, flags, init, out); break;
    default:  // 4 blocks per wave-iteration, one packed tree, workgroup lock-step per group
      hipLaunchKernelGGL(crc_pack4k_kernel<1>, grid, block, 0, s, d_tables, base, stride, nblk, flags, init, out);
      break;
  }
#undef PDB_FAST
#undef PDB_TEAM
  return hipGetLastError();
}

hipError_t launch_desc(const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                       const pdb_blk* blk, uint64_t nblk, uint32_t flags, int mode,
                       const uint32_t* expected, uint32_t* out, uint8_t* ok, uint32_t* nbad,
                       hipStream_t s) {
  if (nblk == 0) return hipSuccess;
  const dim3 grid(grid_for(g, nblk)), block(kThreads);
  const DescSrc src{base, blk, flags};
  if (mode == kModeOut && g_fast_variant == 8)  // A/B: static strided assignment
    hipLaunchKernelGGL((crc_stream_kernel<DescSrc, OutSink, 0, false>), grid, block, 0, s, d_tables, src,
                       nblk, OutSink{out, flags});
  else if (mode == kModeOut)
    hipLaunchKernelGGL((crc_stream_kernel<DescSrc, OutSink, 0, true>), grid, block, 0, s, d_tables, src, nblk,
                       OutSink{out, flags});
  else
    hipLaunchKernelGGL((crc_stream_kernel<DescSrc, VerifySink, 0, true>), grid, block, 0, s, d_tables, src, nblk,
                       VerifySink{expected, ok, nbad, flags});
  return hipGetLastError();
}

hipError_t launch_sst(const LaunchGeom& g, const uint32_t* d_tables, uint8_t* buf, uint64_t buf_len,
                      const pdb_block_handle* h, uint64_t n, bool seal, uint8_t* ok, uint32_t* nbad,
                      hipStream_t s) {
  (void)buf_len;
  if (n == 0) return hipSuccess;
  const dim3 grid(grid_for(g, n)), block(kThreads);
  const SstSrc src{buf, h};
  if (seal)
    hipLaunchKernelGGL((crc_stream_kernel<SstSrc, SealSink, 0, true>), grid, block, 0, s, d_tables, src, n,
                       SealSink{});
  else
    hipLaunchKernelGGL((crc_stream_kernel<SstSrc, SstVerifySink, 0, true>), grid, block, 0, s, d_tables, src, n,
                       SstVerifySink{ok, nbad});
  return hipGetLastError();
}

hipError_t launch_read_stream(const uint8_t* base, uint64_t nbytes, uint32_t* out, hipStream_t s) {
  const uint64_t n16 = nbytes / 16;
  hipLaunchKernelGGL(read_stream_kernel, dim3(256 * 16), dim3(256), 0, s,
                     reinterpret_cast<const u32x4*>(base), n16, out);
  return hipGetLastError();
}

hipError_t launch_read_pattern4k(const LaunchGeom& g, const uint8_t* base, uint64_t nblk,
                                 int variant, uint32_t* out, hipStream_t s) {
  const dim3 grid(g.grid), block(kThreads);
#define PDB_RP(P, D, A) \
  hipLaunchKernelGGL((read_pattern4k_kernel<P, D, A>), grid, block, 0, s, base, nblk, out)
  switch (variant) {
    case 1: PDB_RP(1, 1, 0); break;
    case 2: PDB_RP(0, 2, 0); break;
    case 3: PDB_RP(1, 2, 0); break;
    case 4: PDB_RP(0, 1, 1); break;
    case 5: PDB_RP(1, 1, 1); break;
    case 6: PDB_RP(1, 4, 0); break;
    case 7: PDB_RP(0, 4, 0); break;
    case 8: PDB_RP(2, 1, 0); break;
    case 9: PDB_RP(2, 2, 0); break;
    // workgroup lock-step (one barrier per iteration), as in the shipped CRC kernels
    case 10: hipLaunchKernelGGL((read_pattern4k_kernel<2, 1, 0, true>), grid, block, 0, s, base, nblk, out); break;
    case 11: hipLaunchKernelGGL((read_pattern4k_kernel<1, 1, 0, true>), grid, block, 0, s, base, nblk, out); break;
    case 12: hipLaunchKernelGGL((read_pattern4k_kernel<2, 4, 0, true>), grid, block, 0, s, base, nblk, out); break;
    case 13: hipLaunchKernelGGL((read_pattern4k_kernel<1, 4, 0, true>), grid, block, 0, s, base, nblk, out); break;
    default: PDB_RP(0, 1, 0); break;
  }
#undef PDB_RP
  return hipGetLastError();
}

hipError_t launch_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset,
                                hipStream_t s) {
  if (nbytes == 0) return hipSuccess;
  uint64_t threads = (nbytes + 7) / 8;
  uint64_t blocks = (threads + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(fill_splitmix_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, dst,
                     nbytes, seed, byte_offset);
  return hipGetLastError();
}

}  // namespace pdb
