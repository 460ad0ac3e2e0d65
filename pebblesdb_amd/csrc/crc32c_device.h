// crc32c_device.h -- device-side building blocks of the gfx950 CRC32C kernels, shared by the
// shipped kernels (crc32c_kernels.hip) and the A/B variants and diagnostics (crc32c_variants.hip).
// Everything is in an anonymous namespace: each translation unit instantiates what it uses.
#pragma once
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

// k = 1..3 bytes (low bytes of lb) in one step: x = c ^ lb, c' = XOR_j T_{k-1-j}[x_j] ^ (x >> 8k)
// -- the slice-by-k step, k lookups in parallel instead of k dependent byte steps.
__device__ __forceinline__ uint32_t stepk(const char* lds, const LaneTabs& lt, uint32_t c, uint32_t lb,
                                          uint32_t k) {
  const uint32_t x = c ^ lb;
  if (k == 1) return lds_u32(lds, __builtin_amdgcn_perm(lt.t0, x, sel_byte(0))) ^ (x >> 8);
  if (k == 2)
    return lds_u32(lds, __builtin_amdgcn_perm(lt.t1, x, sel_byte(0))) ^
           lds_u32(lds, __builtin_amdgcn_perm(lt.t0, x, sel_byte(1))) ^ (x >> 16);
  return xor3(lds_u32(lds, __builtin_amdgcn_perm(lt.t2, x, sel_byte(0))),
              lds_u32(lds, __builtin_amdgcn_perm(lt.t1, x, sel_byte(1))),
              lds_u32(lds, __builtin_amdgcn_perm(lt.t0, x, sel_byte(2)))) ^ (x >> 24);
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

// Tree-level operators for the packed / row trees: level l = shift(16 << l) from the single-copy
// slots 0..5 (QuadTree below replaces levels 0 and 1 with replicated, conflict-free copies)
struct SlotTree {
  __device__ __forceinline__ uint32_t op(const char* lds, uint32_t l, uint32_t c, uint32_t y) const {
    return shift_op_x(lds, l, c, y);
  }
};

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
// Loads are issued in batches of 8 per thread before their LDS stores, so staging costs ~2 L2
// round trips instead of one per element (it is most of a small launch's time: the scalar
// Extend path launches one block).
// kQuadTree: slots 0..5 hold the quad-transposed tree's operators {1024, 2048, 64, 128, 256, 512}
// (catalog 6, 7, 2, 3, 4, 5) instead of kTree .. kTree + 5.
template <int kTree, int kHorner, int kSlot7 = -1, bool kSkipSlot5 = false, bool kQuadTree = false>
__device__ __forceinline__ void stage_tables(char* lds, const uint32_t* __restrict__ tabs) {
  constexpr uint32_t kMain = 4u * 256u * 8u;  // 16-B stores of the replicated T0..T3
  for (uint32_t i0 = 0; i0 < kMain; i0 += 8u * blockDim.x) {
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = i0 + threadIdx.x + j * blockDim.x;
      v[j] = i < kMain ? tabs[(i >> 11) * 256u + ((i >> 3) & 255u)] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = i0 + threadIdx.x + j * blockDim.x;
      const uint32_t k = i >> 11, b = (i >> 3) & 255u, part = i & 7u;
      const uint32_t addr = ((k >> 1) << 16) | (b << 8) | ((k & 1u) << 7) | (part << 4);
      if (i < kMain) *reinterpret_cast<u32x4*>(lds + addr) = u32x4{v[j], v[j], v[j], v[j]};
    }
  }
  const u32x4* cat = reinterpret_cast<const u32x4*>(tabs + 1024);
  constexpr uint32_t nslots = kSlot7 >= 0 ? 8u : (kHorner >= 0 ? 7u : 6u);
  constexpr uint32_t kCat = nslots * 256u;
  auto src_of = [](uint32_t slot) -> uint32_t {
    if (kQuadTree && slot < 6) return slot < 2 ? PDB_CAT_S1024 + slot : slot;
    return slot < 6 ? kTree + slot : (slot == 6 ? static_cast<uint32_t>(kHorner) : static_cast<uint32_t>(kSlot7));
  };
  for (uint32_t i0 = 0; i0 < kCat; i0 += 4u * blockDim.x) {
    u32x4 c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = i0 + threadIdx.x + j * blockDim.x;
      const bool use = i < kCat && !(kSkipSlot5 && (i >> 8) == 5);
      c[j] = use ? cat[src_of(i >> 8) * 256u + (i & 255u)] : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = i0 + threadIdx.x + j * blockDim.x;
      const bool use = i < kCat && !(kSkipSlot5 && (i >> 8) == 5);
      if (use) *reinterpret_cast<u32x4*>(lds + PDB_MAIN_BYTES + i * 16u) = c[j];
    }
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
// kNT: non-temporal (streaming) policy.  With kNP = 4 every load instruction reads 1 KiB
// contiguous, and nt loads of that shape read ~12 % faster than any default-policy pattern
// (`read_pattern4k` variants 18/21 vs 12: 6.96 vs 6.22 TB/s); at a 32-B lane stride (kNP = 2)
// nt gains nothing.
template <int kNP, bool kNT = false>
__device__ __forceinline__ void load4k(u32x4 (&v)[4], const uint8_t* base, uint64_t stride, uint64_t b,
                                       uint32_t lane) {
  constexpr uint32_t P = 64u / kNP, gap = 4096u / kNP, per = 4u / kNP;
  const uint8_t* blk = base + b * stride + lane * P;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u32x4* q = reinterpret_cast<const u32x4*>(blk + (i / per) * gap + (i % per) * 16u);
    if constexpr (kNT)
      v[i] = __builtin_nontemporal_load(q);
    else
      v[i] = *q;
  }
}


// ---- fixed-stride batch, 4-KiB packed-tree path ------------------------------------------------
// Same per-block loads and chains as crc_fast4k_kernel<2,1> (64 lanes per block, two 32-B pieces
// per lane), but a wave hashes 4 blocks back to back and folds their 4 x 64 lane partials in ONE
// packed tree: level 0 pairs lanes (2m, 2m+1) of blocks {0,1} and then {2,3} with every lane
// doing useful work, level 1 pairs quads of all 4 blocks in one full-wave round, levels 2-5 run
// once for all 4 blocks.  7 shift operations per 4 blocks instead of 24.
__device__ __forceinline__ uint32_t sel(bool c, uint32_t a, uint32_t b) { return c ? a : b; }

// Returns block (lane & 3)'s raw state in lanes 0..3.
template <bool kL5Twice = false, class TO = SlotTree>
__device__ __forceinline__ uint32_t tree4_packed(const char* lds, uint32_t u, uint32_t p0, uint32_t p1,
                                                 uint32_t p2, uint32_t p3, const TO& to = TO{}) {
  const bool odd = u & 1u;
  // level 0 (shift 32): even lane 2m -> block 0/2 pair m, odd lane 2m+1 -> block 1/3 pair m
  const uint32_t p0n = __builtin_amdgcn_update_dpp(0u, p0, 0x101, 0xF, 0xF, false);  // p0[L+1]
  const uint32_t p1p = __builtin_amdgcn_update_dpp(0u, p1, 0x111, 0xF, 0xF, false);  // p1[L-1]
  const uint32_t r0 = to.op(lds, 0, sel(odd, p1p, p0), sel(odd, p1, p0n));
  const uint32_t p2n = __builtin_amdgcn_update_dpp(0u, p2, 0x101, 0xF, 0xF, false);
  const uint32_t p3p = __builtin_amdgcn_update_dpp(0u, p3, 0x111, 0xF, 0xF, false);
  const uint32_t r1 = to.op(lds, 0, sel(odd, p3p, p2), sel(odd, p3, p2n));
  // level 1 (shift 64): lane 4j+r -> block r pair j.  r<2 reads r0 at L, L+2; r>=2 reads r1 at L-2, L
  const bool hi = u & 2u;
  const uint32_t r0n = __builtin_amdgcn_update_dpp(0u, r0, 0x102, 0xF, 0xF, false);  // r0[L+2]
  const uint32_t r1p = __builtin_amdgcn_update_dpp(0u, r1, 0x112, 0xF, 0xF, false);  // r1[L-2]
  uint32_t v = to.op(lds, 1, sel(hi, r1p, r0), sel(hi, r1, r0n));
  // levels 2..5: lane 4j+r holds block r; pair (L, L + 4*2^(k-2))
  uint32_t y = __builtin_amdgcn_update_dpp(0u, v, 0x104, 0xF, 0xF, false);  // row_shl:4
  if ((u & 4u) == 0) v = shift_op_x(lds, 2, v, y);
  y = __builtin_amdgcn_update_dpp(0u, v, 0x108, 0xF, 0xF, false);  // row_shl:8
  if ((u & 12u) == 0) v = shift_op_x(lds, 3, v, y);
  y = __builtin_amdgcn_ds_swizzle(v, 0x401F);  // lane ^ 16
  if ((u & 28u) == 0) v = shift_op_x(lds, 4, v, y);
  y = __shfl_down(v, 32, 64);
  if ((u & 60u) == 0) {
    if constexpr (kL5Twice)  // slot 5 left free (LDS scratch): shift 2P = shift P twice
      v = shift_op_x(lds, 4, shift_op(lds, 4, v), y);
    else
      v = shift_op_x(lds, 5, v, y);
  }
  return v;
}

// The same packed fold for 8 blocks (partials 16 B apart in every lane): level 0 pairs lanes of
// blocks (0,1), (2,3), (4,5), (6,7) (4 full-wave ops), level 1 quads of blocks 0..3 and 4..7 (2 ops),
// level 2 interleaves the two halves so that lane 8j + b holds block b (1 op), levels 3..5 once
// for all 8 blocks: 10 shift operations per 8 blocks instead of 14.  Block b's raw state ends in
// lane b (b = 0..7).
template <class TO = SlotTree>
__device__ __forceinline__ uint32_t tree8_packed(const char* lds, uint32_t u, const uint32_t (&p)[8], const TO& to = TO{}) {
  const bool odd = u & 1u, hi = u & 2u, h4 = u & 4u;
  uint32_t r[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // level 0 (shift 16): even lane 2m -> block 2k pair m, odd -> 2k+1
    const uint32_t pn = __builtin_amdgcn_update_dpp(0u, p[2 * k], 0x101, 0xF, 0xF, false);      // p[2k][L+1]
    const uint32_t pp = __builtin_amdgcn_update_dpp(0u, p[2 * k + 1], 0x111, 0xF, 0xF, false);  // p[2k+1][L-1]
    r[k] = to.op(lds, 0, sel(odd, pp, p[2 * k]), sel(odd, p[2 * k + 1], pn));
  }
  uint32_t v[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {  // level 1 (shift 32): lane 4j + q -> block 4h + q, quad j
    const uint32_t rn = __builtin_amdgcn_update_dpp(0u, r[2 * h], 0x102, 0xF, 0xF, false);      // [L+2]
    const uint32_t rp = __builtin_amdgcn_update_dpp(0u, r[2 * h + 1], 0x112, 0xF, 0xF, false);  // [L-2]
    v[h] = to.op(lds, 1, sel(hi, rp, r[2 * h]), sel(hi, r[2 * h + 1], rn));
  }
  // level 2 (shift 64): lane 8j + q (q < 4) from v0 at L, L+4; lane 8j + 4 + q from v1 at L-4, L
  const uint32_t vn = __builtin_amdgcn_update_dpp(0u, v[0], 0x104, 0xF, 0xF, false);  // v0[L+4]
  const uint32_t vp = __builtin_amdgcn_update_dpp(0u, v[1], 0x114, 0xF, 0xF, false);  // v1[L-4]
  uint32_t w = shift_op_x(lds, 2, sel(h4, vp, v[0]), sel(h4, v[1], vn));
  // levels 3..5: lane 8j + b holds block b; pair (L, L + 8 * 2^(k-3))
  uint32_t y = __builtin_amdgcn_update_dpp(0u, w, 0x108, 0xF, 0xF, false);  // row_shl:8
  if ((u & 8u) == 0) w = shift_op_x(lds, 3, w, y);
  y = __builtin_amdgcn_ds_swizzle(w, 0x401F);  // lane ^ 16
  if ((u & 24u) == 0) w = shift_op_x(lds, 4, w, y);
  y = __shfl_down(w, 32, 64);
  if ((u & 56u) == 0) w = shift_op_x(lds, 5, w, y);
  return w;
}


// Lane partial of one 4-KiB block.  kNP = 2: two 32-B pieces (at 32l and 2048+32l) folded with
// shift 2048 (slot 6), partials 32 B apart.  kNP = 4: four 16-B pieces at 16l + 1024j, four
// 4-word chains folded as shift2048(shift1024(x0)^x1) ^ (shift1024(x2)^x3) (slots 6, 7), partials
// 16 B apart.
template <int kNP = 2>
__device__ __forceinline__ uint32_t partial4k(const char* lds, const LaneTabs& lt, uint32_t c0,
                                              const u32x4 (&v)[4]) {
  if constexpr (kNP == 4) {
    uint32_t x0 = c0 ^ v[0].x, x1 = v[1].x, x2 = v[2].x, x3 = v[3].x;
    const uint32_t d0[4] = {v[0].x, v[0].y, v[0].z, v[0].w}, d1[4] = {v[1].x, v[1].y, v[1].z, v[1].w};
    const uint32_t d2[4] = {v[2].x, v[2].y, v[2].z, v[2].w}, d3[4] = {v[3].x, v[3].y, v[3].z, v[3].w};
#pragma unroll
    for (int i = 1; i <= 4; ++i) {
      x0 = step4x(lds, lt, x0, i < 4 ? d0[i] : 0u);
      x1 = step4x(lds, lt, x1, i < 4 ? d1[i] : 0u);
      x2 = step4x(lds, lt, x2, i < 4 ? d2[i] : 0u);
      x3 = step4x(lds, lt, x3, i < 4 ? d3[i] : 0u);
    }
    const uint32_t a = shift_op_x(lds, PDB_SLOT_HORNER, x0, x1);
    const uint32_t b = shift_op_x(lds, PDB_SLOT_HORNER, x2, x3);
    return shift_op_x(lds, PDB_SLOT_HORNER + 1, a, b);
  }
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

// ---- lane-quarter table image: conflict-free tables AND Horner operators ---------------------
// The 32-replica T0..T3 image above makes every table lookup conflict-free but takes 128 KiB, so
// the shift operators live in single copies and a 64-lane operator lookup costs ~3 extra LDS cycles
// of bank conflicts (4 random bytes -> 32 banks).  In the lane-quarter image (the record kernel's,
// crc32c_lanespan.h) lookup instruction i sends lane quarter q = (lane >> 3) & 3 to table
// k = (q + i) & 3, replica lane & 7: the four quarters of each 32-lane group read four tables in
// four disjoint bank ranges, so 8 replicas are conflict-free -- 32 KiB per four tables.  An operator
// (4 sub-tables indexed by the 4 state bytes) is looked up the same way: its sub-table 3 - k sits
// where T_k does, so the T lookup's address byte and byte selector serve it unchanged.  64-KiB
// images of 256 entry blocks (entry b at b << 8, the state byte placed by one v_perm):
//   image 0 [0, 64 KiB):       T_k replica r at dword k*8 + r; shift 1024 sub-table 3-k at 32 + k*8 + r
//   image 1 [64 KiB, 128 KiB): shift 2048 sub-table 3-k at dword k*8 + r  (dwords 32..63 unused)
// and the tree operators (single copies, fewer lanes active per lookup) in slots 0..5 of the OPS
// region as before.
struct QuadTabs {
  uint32_t t[4], s[4];  // address byte 0 (table slot, replica) and byte selector (byte 3 - k) of lookup i
  uint32_t g[4];        // t | 0x10000: image 1 (the immediate offset of a ds_read stops at 64 KiB)
};

__device__ __forceinline__ QuadTabs quad_tabs(uint32_t u) {
  const uint32_t r = u & 7u, q = (u >> 3) & 3u;
  QuadTabs qt;
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
    const uint32_t k = (q + i) & 3u, a = (k * 8u + r) << 2;
    qt.t[i] = a;
    qt.s[i] = sel_byte(3u - k);
    qt.g[i] = 0x10000u | a;
  }
  return qt;
}

// x' = shift(x, 4 bytes) ^ wnext on the lane-quarter image (the same value as the LaneTabs form)
__device__ __forceinline__ uint32_t step4x(const char* lds, const QuadTabs& qt, uint32_t x, uint32_t wnext) {
  const uint32_t a0 = __builtin_amdgcn_perm(qt.t[0], x, qt.s[0]);
  const uint32_t a1 = __builtin_amdgcn_perm(qt.t[1], x, qt.s[1]);
  const uint32_t a2 = __builtin_amdgcn_perm(qt.t[2], x, qt.s[2]);
  const uint32_t a3 = __builtin_amdgcn_perm(qt.t[3], x, qt.s[3]);
  return xor3(xor3(lds_u32(lds, a0), lds_u32(lds, a1), lds_u32(lds, a2)), lds_u32(lds, a3), wnext);
}

// shift(c, D) ^ y through a replicated operator whose sub-tables sit at `base` (+ `off`)
template <uint32_t off>
__device__ __forceinline__ uint32_t op_q(const char* lds, const uint32_t (&base)[4], const uint32_t (&s)[4], uint32_t c,
                                         uint32_t y) {
  const char* l = lds + off;  // folded into the ds_read immediate offset
  const uint32_t a0 = __builtin_amdgcn_perm(base[0], c, s[0]);
  const uint32_t a1 = __builtin_amdgcn_perm(base[1], c, s[1]);
  const uint32_t a2 = __builtin_amdgcn_perm(base[2], c, s[2]);
  const uint32_t a3 = __builtin_amdgcn_perm(base[3], c, s[3]);
  return xor3(xor3(lds_u32(l, a0), lds_u32(l, a1), lds_u32(l, a2)), lds_u32(l, a3), y);
}

// One slice-by-4 step c' = shift(c ^ w, 4) (the head words of the stream kernel)
__device__ __forceinline__ uint32_t step4(const char* lds, const QuadTabs& qt, uint32_t c, uint32_t w) {
  return step4x(lds, qt, c ^ w, 0u);
}

// stepk on the lane-quarter image: k = 1..3 leading bytes, every lane reading table k-1-j through
// its own replica (a wave-uniform head: the lanes share the entry, no conflicts)
__device__ __forceinline__ uint32_t stepk(const char* lds, const QuadTabs& qt, uint32_t c, uint32_t lb, uint32_t k) {
  const uint32_t x = c ^ lb, r = qt.t[0] & 0x1Cu;  // (lane & 7) << 2
  auto T = [&](uint32_t tab, uint32_t byte) { return lds_u32(lds, (((x >> (8u * byte)) & 0xFFu) << 8) | (tab << 5) | r); };
  if (k == 1) return T(0, 0) ^ (x >> 8);
  if (k == 2) return T(1, 0) ^ T(0, 1) ^ (x >> 16);
  return xor3(T(2, 0), T(1, 1), T(0, 2)) ^ (x >> 24);
}

// Tree levels 0 and 1 (shift 16 / 32, the levels every lane works in) from replicated copies in
// image 1 at byte offset kOff0 / kOff1 of an entry block (-1: the single-copy slot)
template <int kOff0, int kOff1>
struct QuadTree {
  const QuadTabs& qt;
  __device__ __forceinline__ uint32_t op(const char* lds, uint32_t l, uint32_t c, uint32_t y) const {
    if constexpr (kOff0 >= 0)
      if (l == 0) return op_q<static_cast<uint32_t>(kOff0)>(lds, qt.g, qt.s, c, y);
    if constexpr (kOff1 >= 0)
      if (l == 1) return op_q<static_cast<uint32_t>(kOff1)>(lds, qt.g, qt.s, c, y);
    return shift_op_x(lds, l, c, y);
  }
};

// shift(c, 1024) ^ y: the Horner fold of 16-B pieces 1 KiB apart, on either image
__device__ __forceinline__ uint32_t horner1024(const char* lds, const LaneTabs&, uint32_t c, uint32_t y) {
  return shift_op_x(lds, PDB_SLOT_HORNER, c, y);
}
__device__ __forceinline__ uint32_t horner1024(const char* lds, const QuadTabs& qt, uint32_t c, uint32_t y) {
  return op_q<128u>(lds, qt.t, qt.s, c, y);
}
// shift(c, 1008): the stream kernel's round chaining (slot 6 of the 32-replica image; image 1)
__device__ __forceinline__ uint32_t round1008(const char* lds, const LaneTabs&, uint32_t c) {
  return shift_op(lds, PDB_SLOT_HORNER, c);
}
__device__ __forceinline__ uint32_t round1008(const char* lds, const QuadTabs& qt, uint32_t c) {
  return op_q<0u>(lds, qt.g, qt.s, c, 0u);
}

// Stage image 0, image 1 (catalog operators kImg1Lo in dwords 0..31 and kImg1Hi in 32..63 of its
// entry blocks: shift 2048 / 1008 for the Horner folds of crc_pack4k_kernel / the stream kernel,
// the tree's level-0 / level-1 operators; -1: none) and the tree operators (catalog kTree ..
// kTree + 5 -> slots 0..5), all of a thread's loads issued before its stores (launch latency
// matters for small batches).
template <int kTree, int kImg1Lo, int kImg1Hi = -1>
__device__ __forceinline__ void stage_tables_q4(char* lds, const uint32_t* __restrict__ tabs) {
  // 16-B quads: q < kRep = replicated quads (part q >> 11: T, shift 1024, image 1 lo, image 1 hi,
  // the absent ones skipped; entry b, table slot k, replicas 4h..4h+3), then 1536 single-copy
  // tree-operator quads
  static_assert(kImg1Lo >= 0 || kImg1Hi < 0, "image 1 fills its low half first");
  constexpr uint32_t kRep = (2u + (kImg1Lo >= 0 ? 1u : 0u) + (kImg1Hi >= 0 ? 1u : 0u)) * 2048u, kAll = kRep + 6u * 256u;
  const u32x4* cat = reinterpret_cast<const u32x4*>(tabs + 1024);
  for (uint32_t i0 = 0; i0 < kAll; i0 += 8u * blockDim.x) {
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = i0 + threadIdx.x + j * blockDim.x;
      if (i < kRep) {
        const uint32_t part = i >> 11, b = (i >> 3) & 255u, k = (i >> 1) & 3u;
        // T_k, or operator sub-table 3 - k (tabs: T0..T3, then the catalog's 4 x 256 per operator)
        const uint32_t cat_id = part == 1 ? PDB_CAT_S1024 : (part == 2 ? static_cast<uint32_t>(kImg1Lo) : static_cast<uint32_t>(kImg1Hi));
        const uint32_t src = part == 0 ? k * 256u + b : 1024u + cat_id * 1024u + (3u - k) * 256u + b;
        const uint32_t x = tabs[src];
        v[j] = u32x4{x, x, x, x};
      } else {
        const uint32_t t = i - kRep;
        v[j] = t < 6u * 256u ? cat[(kTree + (t >> 8)) * 256u + (t & 255u)] : u32x4{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = i0 + threadIdx.x + j * blockDim.x;
      if (i < kRep) {
        const uint32_t part = i >> 11, b = (i >> 3) & 255u, k = (i >> 1) & 3u, h = i & 1u;
        const uint32_t addr = (part >= 2 ? 0x10000u : 0u) | (b << 8) | ((part & 1u) ? 128u : 0u) | (k << 5) | (h << 4);
        *reinterpret_cast<u32x4*>(lds + addr) = v[j];
      } else if (i < kAll) {
        *reinterpret_cast<u32x4*>(lds + PDB_MAIN_BYTES + (i - kRep) * 16u) = v[j];
      }
    }
  }
}

// partial4k<4> on the lane-quarter image: four 4-word chains, Horner folds through the replicated
// shift 1024 / shift 2048.  kDeferF: the chains stop with their last word still unshifted (3 table
// steps instead of 4): the final table step F (shift 4) commutes with every shift operator of the
// folds and the tree, so the caller applies it ONCE to the tree's result -- 1 step per 4 blocks
// instead of 16 per lane per block (-18 % LDS lookups, -15 % VALU per block).
template <bool kDeferF = true>
__device__ __forceinline__ uint32_t partial4k_q(const char* lds, const QuadTabs& qt, uint32_t c0, const u32x4 (&v)[4]) {
  uint32_t x0 = c0 ^ v[0].x, x1 = v[1].x, x2 = v[2].x, x3 = v[3].x;
  const uint32_t d0[4] = {v[0].x, v[0].y, v[0].z, v[0].w}, d1[4] = {v[1].x, v[1].y, v[1].z, v[1].w};
  const uint32_t d2[4] = {v[2].x, v[2].y, v[2].z, v[2].w}, d3[4] = {v[3].x, v[3].y, v[3].z, v[3].w};
#pragma unroll
  for (int i = 1; i <= (kDeferF ? 3 : 4); ++i) {
    x0 = step4x(lds, qt, x0, i < 4 ? d0[i] : 0u);
    x1 = step4x(lds, qt, x1, i < 4 ? d1[i] : 0u);
    x2 = step4x(lds, qt, x2, i < 4 ? d2[i] : 0u);
    x3 = step4x(lds, qt, x3, i < 4 ? d3[i] : 0u);
  }
  const uint32_t a = horner1024(lds, qt, x0, x1);
  const uint32_t b = horner1024(lds, qt, x2, x3);
  return op_q<0u>(lds, qt.g, qt.s, a, b);  // shift 2048
}

// ---- fixed-stride batch, 4-KiB path (BASELINE configs 2 and 4) -------------------------------
// len == 4096, base and stride 16-B aligned.  One wave per block; lane u owns the four 16-B pieces
// at 16u + 1024j (j = 0..3), so each of a block's 4 load instructions reads 1 KiB contiguous,
// issued non-temporal, and the pieces are 4 independent chains folded by partial4k_q (the
// lane-quarter image: the Horner operators conflict-free, +4-7 % over partial4k<4>).  A wave
// hashes 4 blocks (g, g+W, g+2W, g+3W; W = waves in the grid), the next block's loads issued before
// the current one is hashed, and folds their 4 x 64 lane partials in ONE tree4_packed.  One
// barrier per 4-block group keeps the workgroup's 16 waves on 16 consecutive blocks (DRAM row
// locality: +8 %).  Results are parked in a register and flushed as one 64-lane
// store per 16 groups.  The A/B variants of this kernel (piece shapes, waves per CU, lock-step
// period, XCD numbering, quad transposes) were diagnostics-library variants until round 4.
// kW: waves per workgroup (one workgroup per CU); 16 shipped, 8 / 12 A/B variants.  kDeferF: one
// table step per 4 blocks after the tree (partial4k_q); false = the round-2 form (A/B).
template <uint32_t kW = kWavesPerWg, bool kDeferF = true>
__global__ __launch_bounds__(64 * kW) void crc_pack4k_kernel(
    const uint32_t* __restrict__ tabs, const uint8_t* __restrict__ base, uint64_t stride,
    uint64_t nblk, uint32_t flags, uint32_t init, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  const uint32_t u = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kW;
  const uint64_t wg_first = static_cast<uint64_t>(blockIdx.x) * kW;
  const uint64_t w = wg_first + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u32x4 buf[4];
  load4k<4, true>(buf, base, stride, w < nblk ? w : nblk - 1, u);  // overlaps the table staging
  stage_tables_q4<PDB_CAT_TREE16, PDB_CAT_S2048, PDB_CAT_TREE16>(lds, tabs);  // image 1 hi: tree level 0
  __syncthreads();
  if (wg_first >= nblk) return;  // workgroup-uniform: every wave of a live workgroup reaches each barrier
  const QuadTabs qt = quad_tabs(u);
  const uint32_t init_raw = (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu;
  const uint32_t c0 = u == 0 ? init_raw : 0u;
  uint32_t res = 0, it = 0;
  uint64_t win0 = w;
  for (uint64_t g = w, gw = wg_first; gw < nblk; g += 4 * nw, gw += 4 * nw) {
    __syncthreads();  // lock step: the CU's 16 waves load 16 consecutive blocks at a time
    uint32_t p[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint64_t bk = g + r * nw;
      u32x4 cur[4] = {buf[0], buf[1], buf[2], buf[3]};
      const uint64_t bn = bk + nw;
      if (bn < nblk) load4k<4, true>(buf, base, stride, bn, u);  // wave-uniform
      p[r] = bk < nblk ? partial4k_q<kDeferF>(lds, qt, c0, cur) : 0u;
    }
    uint32_t v = tree4_packed(lds, u, p[0], p[1], p[2], p[3], QuadTree<128, -1>{qt});
    if constexpr (kDeferF) v = step4x(lds, qt, v, 0u);  // F: the chains' last words
    // lane 4j+r of the 64-block window holds block (window + (4j+r)*nw): move lanes 0..3's
    // results up by 4*(group mod 16) with one bpermute, park, flush every 16 groups.
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

// Sources: get(i) = the descriptor of block i.  load(i) / finish(raw) split it so a kernel can
// issue block i's descriptor load one block ahead and only touch the value when the block is
// due: load() is a vector load into VGPRs (never an SMEM load, whose lgkmcnt would also stall the
// kernel's LDS lookups) and finish() makes the fields wave-uniform.
struct FixedSrc {
  const uint8_t* base;
  uint64_t stride;
  uint32_t len;
  uint32_t init_raw;
  using Raw = uint64_t;
  __device__ __forceinline__ Raw load(uint64_t i) const { return i; }
  __device__ __forceinline__ Raw load_cached(uint64_t i) const { return i; }
  __device__ __forceinline__ BlkDesc finish(Raw i) const { return {base + i * stride, len, init_raw}; }
  __device__ __forceinline__ BlkDesc get(uint64_t i) const { return finish(i); }
  __device__ __forceinline__ BlkDesc lane(Raw i) const { return finish(i); }  // per-lane fields
  // (a fixed stride's length is known to the host: no long-block lane)
  __device__ __forceinline__ bool long_export(uint64_t, const BlkDesc&, uint32_t, uint32_t) const { return false; }
  __device__ __forceinline__ bool long_export_cold(uint64_t, const BlkDesc&, uint32_t, uint32_t) const { return false; }
};

// Descriptor fields are loaded by every lane from one address, so the compiler sees per-lane
// (VGPR) values; readfirstlane makes them wave-uniform SGPRs, which keeps the block geometry
// (rounds, chains, head) on scalar branches instead of exec-masked divergent code.
__device__ __forceinline__ uint64_t uniform64(uint32_t lo, uint32_t hi) {
  const uint32_t l = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(lo));
  const uint32_t h = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(hi));
  return (static_cast<uint64_t>(h) << 32) | l;
}

// The long-block lane (crc32c_internal.h): export block i (p, n bytes, seed init_raw; wave-uniform
// arguments, every lane calling) when it has at least min_bytes and the scratch at `lane` has room:
// lane 0 reserves a record and np = ceil(n / 4096) pieces with one compare-and-swap loop (no
// reservation is ever left half-made, so every reserved piece is written), then the wave writes the
// record and the piece list.  False: the caller hashes the block itself.  (A batch kernel carries
// the scratch base alone: the layout is fixed, and every SGPR counts in these kernels.)
__device__ __forceinline__ bool long_export(uint8_t* lane, uint32_t min_bytes, uint64_t i, uintptr_t p, uint32_t n,
                                            uint32_t init_raw, uint32_t u) {
  if (!lane || n < min_bytes) return false;
  unsigned long long* hdr = reinterpret_cast<unsigned long long*>(lane);
  const uint32_t m = (n - 1u) >> 12, np = m + 1u, h = n - (m << 12);
  unsigned long long got = ~0ull;
  if (u == 0) {
    unsigned long long old = __hip_atomic_load(hdr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      if ((old >> 40) >= kLongRecCap || (old & kLongPieceMask) + np > kLongPieceCap) break;
      if (__hip_atomic_compare_exchange_strong(hdr, &old, old + ((1ull << 40) | np), __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        got = old;
        break;
      }
    }
  }
  got = uniform64(__builtin_amdgcn_readlane(static_cast<uint32_t>(got), 0),
                  __builtin_amdgcn_readlane(static_cast<uint32_t>(got >> 32), 0));
  if (got == ~0ull) return false;
  const uint32_t slot = static_cast<uint32_t>(got >> 40), q0 = static_cast<uint32_t>(got & kLongPieceMask);
  LongRec* rec = reinterpret_cast<LongRec*>(lane + kLongRecOff);
  LongPiece* piece = reinterpret_cast<LongPiece*>(lane + kLongPieceOff);
  if (u == 0) rec[slot] = LongRec{i, static_cast<uint64_t>(p), n, init_raw, q0, np};
  for (uint32_t k = u; k < np; k += 64u)
    piece[q0 + k] = k ? LongPiece{static_cast<uint64_t>(p) + h + 4096ull * (k - 1u), 4096u, 0u}
                      : LongPiece{static_cast<uint64_t>(p), h, 1u};
  return true;
}

// The same as a real call, made only for a block already known to be long (the caller tests the
// length inline): inlined into the sstable-sized kernel's drain, the export changes the register
// allocation of the whole kernel (more spills: verify -1 %, in-place seal -0.4 % on one box,
// tools/ab_lane.sh, profiles/r06/ab_lane/); as a call on that cold path it costs nothing.  (In the
// stream kernel's block loop any call site costs C3 6-7 %: it keeps the inline form.)
__device__ __attribute__((noinline)) bool long_export_call(uint8_t* lane, uint32_t min_bytes, uint64_t i, uintptr_t p,
                                                           uint32_t n, uint32_t init_raw, uint32_t u) {
  return long_export(lane, min_bytes, i, p, n, init_raw, u);
}

struct DescSrc {
  const uint8_t* base;
  const pdb_blk* blk;
  uint32_t flags;
  uint8_t* long_lane = nullptr;  // the long-block lane's scratch (null: off)
  // inline (the stream kernel's block loop: a call site there costs C3 6-7 %, tools/ab_lane.sh)
  __device__ __forceinline__ bool long_export(uint64_t i, const BlkDesc& d, uint32_t u, uint32_t min_bytes) const {
    return pdb::long_export(long_lane, min_bytes, i, reinterpret_cast<uintptr_t>(d.p), d.n, d.init_raw, u);
  }
  // as a call, for a block already known to be deferred (the sstable-sized kernel's drain)
  __device__ __forceinline__ bool long_export_cold(uint64_t i, const BlkDesc& d, uint32_t u, uint32_t min_bytes) const {
    return long_lane && d.n >= min_bytes &&
           pdb::long_export_call(long_lane, min_bytes, i, reinterpret_cast<uintptr_t>(d.p), d.n, d.init_raw, u);
  }
  using Raw = u32x4;  // pdb_blk {off lo, off hi, len, init}
  __device__ __forceinline__ Raw load(uint64_t i) const {
    // 8-B alignment is all pdb_blk guarantees: a 4-B-aligned 16-B load
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4a4*>(blk + i));
  }
  // the same, cached (a consumer that re-reads a batch's descriptors: crc_lanespan_kernel)
  __device__ __forceinline__ Raw load_cached(uint64_t i) const {
    return *reinterpret_cast<const u32x4a4*>(blk + i);
  }
  __device__ __forceinline__ BlkDesc finish(const Raw& r) const {
    const uint32_t len = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(r.z));
    const uint32_t init = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(r.w));
    return {base + uniform64(r.x, r.y), len, (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu};
  }
  __device__ __forceinline__ BlkDesc get(uint64_t i) const { return finish(load(i)); }
  __device__ __forceinline__ BlkDesc lane(const Raw& r) const {  // per-lane fields (no readfirstlane)
    return {base + ((static_cast<uint64_t>(r.y) << 32) | r.x), r.z, (flags & PDB_CRC_USE_INIT) ? ~r.w : 0xFFFFFFFFu};
  }
  // block i's offset and length (the byte-balanced split, bal_bound)
  __device__ __forceinline__ uint64_t off(uint64_t i) const {
    typedef __attribute__((address_space(1))) const uint64_t g_u64_;
    return *reinterpret_cast<g_u64_*>(reinterpret_cast<uintptr_t>(&blk[i].off));
  }
  __device__ __forceinline__ uint32_t len(uint64_t i) const {
    typedef __attribute__((address_space(1))) const uint32_t g_u32_;
    return *reinterpret_cast<g_u32_*>(reinterpret_cast<uintptr_t>(&blk[i].len));
  }
};

// Byte-balanced workgroup boundaries for descriptor lists (C3: Zipf sizes): workgroup g's first
// block is the first block whose offset reaches g/G of the list's span (off[0] .. off[n-1] +
// len[n-1]), searched 64 ways per step by one wave (3 dependent loads for C3's ~4800-block
// windows), and CLAMPED to within D - 1 blocks of the count split n g / G, D = floor(n / 2G).
// Consecutive count splits are >= 2D - 2 apart, so the boundaries are non-decreasing in g and the
// workgroups partition [0, n) whatever the list holds; on a packed ascending list (every C3 list)
// each workgroup gets ~1/G of the bytes instead of 1/G of the blocks.  All 64 lanes must be
// active; the result is wave-uniform.
template <class Src>
__device__ __forceinline__ uint64_t bal_bound(const Src& src, uint64_t n, uint64_t g, uint64_t G, uint32_t u) {
  const uint64_t cs = n * g / G;
  const uint64_t D = n / (2 * G);
  if (g == 0 || g >= G || D < 2) return cs;
  const uint64_t o0 = src.off(0), oe = src.off(n - 1) + src.len(n - 1);
  if (oe <= o0) return cs;
  const uint64_t span = oe - o0;
  const uint64_t t = o0 + span / G * g + span % G * g / G;  // o0 + span g / G without overflow
  uint64_t lo = cs - (D - 1), hi = cs + (D - 1);              // the boundary lies in [lo, hi]
  while (lo < hi) {
    const uint64_t step = (hi - lo + 63u) / 64u;
    const uint64_t sidx = lo + u * step;
    const bool valid = sidx < hi;
    const uint64_t o = src.off(valid ? sidx : lo);
    const uint64_t m = __builtin_amdgcn_ballot_w64(valid && o >= t);
    if (m & 1ull) break;  // block lo already reaches t
    if (m == 0) {
      lo += ((hi - lo - 1u) / step) * step + 1u;  // past the last sample
    } else {
      const uint64_t k = static_cast<uint64_t>(__builtin_ctzll(m));
      hi = lo + k * step;
      lo += (k - 1u) * step + 1u;
    }
  }
  return lo;
}

// sstable handle: CRC over contents || type (table/table_builder.cc:197-198; format.cc:98).
// A handle whose block + 5-byte trailer does not fit the buffer (ReadBlock's "truncated block
// read", table/format.cc:84-87 -- a corrupt index must not make the kernel read or write outside
// the image) maps to {buf, 0, 0}: nothing is hashed, and init_raw 0 (never Value()'s seed) tells
// the sst sinks to report the block bad (verify) or leave it alone (seal).
struct SstSrc {
  uint8_t* buf;
  const pdb_block_handle* h;
  uint64_t len;  // image bytes
  uint8_t* long_lane = nullptr;
  // inline (the stream kernel's block loop: a call site there costs C3 6-7 %, tools/ab_lane.sh)
  __device__ __forceinline__ bool long_export(uint64_t i, const BlkDesc& d, uint32_t u, uint32_t min_bytes) const {
    return pdb::long_export(long_lane, min_bytes, i, reinterpret_cast<uintptr_t>(d.p), d.n, d.init_raw, u);
  }
  // as a call, for a block already known to be deferred (the sstable-sized kernel's drain)
  __device__ __forceinline__ bool long_export_cold(uint64_t i, const BlkDesc& d, uint32_t u, uint32_t min_bytes) const {
    return long_lane && d.n >= min_bytes &&
           pdb::long_export_call(long_lane, min_bytes, i, reinterpret_cast<uintptr_t>(d.p), d.n, d.init_raw, u);
  }
  using Raw = u32x4;  // pdb_block_handle {offset lo, hi, size lo, hi}
  __device__ __forceinline__ Raw load(uint64_t i) const {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4a4*>(h + i));
  }
  __device__ __forceinline__ BlkDesc make(uint64_t off, uint64_t size) const {
    // (the 12-wave verify spills 2 VGPRs in its prologue, ~1.5 MB of scratch writes per 1 M-block
    // launch: uniform values the compiler keeps as VGPR copies.  Writing this check as off + size <=
    // len - 5 without the len >= 5 term took them to 1 and cost the 12-wave seal 1.2 %, both orders on
    // one box (tools/ab_lane.sh, profiles/r06/ab_lane/ab_spill.log): not kept.)
    const bool ok = len >= 5 && off <= len - 5 && size <= len - 5 - off && size < 0xFFFFFFFFull;
    return ok ? BlkDesc{buf + off, static_cast<uint32_t>(size) + 1u, 0xFFFFFFFFu} : BlkDesc{buf, 0u, 0u};
  }
  __device__ __forceinline__ BlkDesc finish(const Raw& r) const { return make(uniform64(r.x, r.y), uniform64(r.z, r.w)); }
  __device__ __forceinline__ BlkDesc get(uint64_t i) const { return finish(load(i)); }
  __device__ __forceinline__ BlkDesc lane(const Raw& r) const {  // per-lane fields (no readfirstlane)
    return make((static_cast<uint64_t>(r.y) << 32) | r.x, (static_cast<uint64_t>(r.w) << 32) | r.z);
  }
};

// The long-block lane's pieces (crc_longpiece_kernel): piece q = {p, n, seeded}; init_raw carries the
// seed the sstable-sized kernel starts a 4096-B piece from (SrcSeeds): 0xFFFFFFFF for a head
// (Value()), 0 for a full piece (raw state 0).  A head of another length takes the kernel's slow path,
// which is Value()-seeded.
struct PieceSrc {
  const LongPiece* piece;
  using Raw = u32x4;  // {p lo, p hi, n, seeded}
  __device__ __forceinline__ Raw load(uint64_t i) const {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(piece + i));
  }
  __device__ __forceinline__ BlkDesc lane(const Raw& r) const {
    return {reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(r.y) << 32) | r.x), r.z, r.w ? 0xFFFFFFFFu : 0u};
  }
  __device__ __forceinline__ bool long_export(uint64_t, const BlkDesc&, uint32_t, uint32_t) const { return false; }
  __device__ __forceinline__ bool long_export_cold(uint64_t, const BlkDesc&, uint32_t, uint32_t) const { return false; }
};

// Start state of a 4096-B block in the sstable-sized kernel: Value()'s seed, or the piece's own.
template <class Src>
struct SrcSeeds {
  static constexpr bool kOn = false;
};
template <>
struct SrcSeeds<PieceSrc> {
  static constexpr bool kOn = true;
};

// The pieces' raw states (leaves of the long-block combine)
struct LeafSink {
  uint32_t* leaf;
  __device__ __forceinline__ void put(uint64_t i, uint32_t raw, const BlkDesc&) const { leaf[i] = raw; }
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
    if (d.init_raw == 0) return;  // invalid handle (SstSrc): nothing to seal
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
    const bool good = d.init_raw != 0 && pdb_unmask(stored) == ~raw;  // init_raw 0: invalid handle
    if (ok) ok[i] = good ? 1 : 0;
    if (!good && nbad) atomicAdd(nbad, 1u);
  }
};

// The seal's trailer words into a compact array (pdb_sst_crc_device, the host seal's staging):
// out[i] = Mask(crc); an invalid handle (SstSrc init_raw 0) leaves out[i] untouched.
struct SstCrcSink {
  uint32_t* out;
  __device__ __forceinline__ void put(uint64_t i, uint32_t raw, const BlkDesc& d) const {
    if (d.init_raw != 0) out[i] = pdb_mask(~raw);
  }
};

// Sink access for crc_sst4k_kernel: pre() issues whatever the sink reads (the stored trailer a
// verify compares with) a group ahead, so put() never waits on a load issued after the next
// group's prefetch; all accesses through global-address-space pointers (the kernel's block
// addresses are integers; a flat access would also count in lgkmcnt and stall LDS lookups).
template <class Sink>
struct SinkOps {
  __device__ static __forceinline__ uint32_t pre(const Sink&, uint64_t, const BlkDesc&) { return 0u; }
  __device__ static __forceinline__ void put(const Sink& k, uint64_t i, uint32_t raw, const BlkDesc& d, uint32_t) {
    k.put(i, raw, d);
  }
};

template <>
struct SinkOps<VerifySink> {  // the expected CRC, loaded a group ahead
  __device__ static __forceinline__ uint32_t pre(const VerifySink& k, uint64_t i, const BlkDesc&) {
    typedef __attribute__((address_space(1))) const uint32_t g_u32_;
    return *reinterpret_cast<g_u32_*>(reinterpret_cast<uintptr_t>(k.expected + i));
  }
  __device__ static __forceinline__ void put(const VerifySink& k, uint64_t i, uint32_t raw, const BlkDesc&,
                                             uint32_t expected) {
    const bool good = finalize(raw, k.flags) == expected;
    if (k.ok) k.ok[i] = good ? 1 : 0;
    if (!good && k.nbad) atomicAdd(k.nbad, 1u);
  }
};

template <>
struct SinkOps<SealSink> {
  __device__ static __forceinline__ uint32_t pre(const SealSink&, uint64_t, const BlkDesc&) { return 0u; }
  __device__ static __forceinline__ void put(const SealSink&, uint64_t, uint32_t raw, const BlkDesc& d, uint32_t) {
    if (d.init_raw == 0) return;  // invalid handle (SstSrc): nothing to seal
    typedef __attribute__((address_space(1))) uint8_t g_u8;
    g_u8* tr = reinterpret_cast<g_u8*>(reinterpret_cast<uintptr_t>(d.p) + d.n);
    const uint32_t m = pdb_mask(~raw);
    tr[0] = static_cast<uint8_t>(m);
    tr[1] = static_cast<uint8_t>(m >> 8);
    tr[2] = static_cast<uint8_t>(m >> 16);
    tr[3] = static_cast<uint8_t>(m >> 24);
  }
};

// Seal with PARKED trailers (sstable-sized kernel, 4-block groups): a wave keeps the trailers of its
// last kRing groups in lanes (lane 4 (g mod kRing) + r: block r of the wave's g-th group) and writes
// each one when its lane slot comes round again, i.e. kRing groups later; the rest at the end.
// kRing = 0: the plain SealSink behaviour (write when hashed).
template <class Sink>
struct SinkPark {
  static constexpr uint32_t kRing = 0;
};
template <uint32_t R>
struct ParkSealSink {};
template <uint32_t R>
struct SinkPark<ParkSealSink<R>> {
  static_assert(R == 1 || R == 2 || R == 4 || R == 8 || R == 16 || R == 32 || R == 64, "ring of lane slots");
  static constexpr uint32_t kRing = R;
};
template <uint32_t R>
struct SinkOps<ParkSealSink<R>> {  // the deferred (slow-path) blocks: written when hashed
  __device__ static __forceinline__ uint32_t pre(const ParkSealSink<R>&, uint64_t, const BlkDesc&) { return 0u; }
  __device__ static __forceinline__ void put(const ParkSealSink<R>&, uint64_t i, uint32_t raw, const BlkDesc& d,
                                             uint32_t) {
    SinkOps<SealSink>::put(SealSink{}, i, raw, d, 0u);
  }
};
__device__ __forceinline__ void write_trailer_word(uintptr_t a, uint32_t m) {
  typedef __attribute__((address_space(1))) uint8_t g_u8;
  g_u8* tr = reinterpret_cast<g_u8*>(a);
  tr[0] = static_cast<uint8_t>(m);
  tr[1] = static_cast<uint8_t>(m >> 8);
  tr[2] = static_cast<uint8_t>(m >> 16);
  tr[3] = static_cast<uint8_t>(m >> 24);
}

template <>
struct SinkOps<SstVerifySink> {
  // the stored trailer word at p + n (any alignment): ONE dword load at its own byte address (the
  // runtime runs shaders in unaligned access mode: the memory pipeline splits it when it crosses a
  // dword, and this is one load per block, off the hashing path).  Round 3 loaded the two aligned
  // dwords and merged them with v_alignbyte: one more register live per block in flight, which in
  // the 12-wave verify (168 VGPRs a lane) spilled -- 6.45 MB of scratch writes per 1 M-block
  // launch against 1.05 MB of `ok` bytes.
  __device__ static __forceinline__ uint32_t pre(const SstVerifySink&, uint64_t, const BlkDesc& d) {
    typedef __attribute__((address_space(1), aligned(1))) const uint32_t g_u32u_;
    return *reinterpret_cast<g_u32u_*>(reinterpret_cast<uintptr_t>(d.p) + d.n);
  }
  __device__ static __forceinline__ void put(const SstVerifySink& k, uint64_t i, uint32_t raw, const BlkDesc& d,
                                             uint32_t stored) {
    const bool good = d.init_raw != 0 && pdb_unmask(stored) == ~raw;  // init_raw 0: invalid handle
    if (k.ok) k.ok[i] = good ? 1 : 0;
    if (!good && k.nbad) atomicAdd(k.nbad, 1u);
  }
  // the ok byte alone (crc_sst4k_kernel's LDS ring of ok bytes, OkRing below)
  __device__ static __forceinline__ uint8_t verdict(const SstVerifySink& k, uint32_t raw, const BlkDesc& d, uint32_t stored) {
    const bool good = d.init_raw != 0 && pdb_unmask(stored) == ~raw;
    if (!good && k.nbad) atomicAdd(k.nbad, 1u);
    return good ? 1 : 0;
  }
};

// Sinks whose per-block byte crc_sst4k_kernel gathers in an LDS ring of 64-block lines and stores
// as one 64-lane byte store per line (OkRing): the verify's ok flags.
template <class Sink>
struct SinkRing {
  static constexpr bool kOn = false;
};
template <>
struct SinkRing<SstVerifySink> {
  static constexpr bool kOn = true;
};

// Rounds of a block of K 32-B pieces: 128 pieces (4 KiB) per round, and the block's last round
// may take up to 64 more as a third chain (piece u + 128 on lane u), so a block of 4 KiB + a few
// bytes -- every real sstable data block: 4171-4175 B with the type byte -- is one round, not a
// full second round for its last 2 pieces.
__device__ __forceinline__ uint32_t rounds32(uint32_t K) {
  const uint32_t r = (K + 63u) >> 7;
  return r ? r : 1u;
}

// Same for the 16-B-piece kernels: 256 pieces per round, up to 64 more as a fifth chain.
__device__ __forceinline__ uint32_t rounds16(uint32_t K) {
  const uint32_t r = (K + 191u) >> 8;
  return r ? r : 1u;
}

// Raw (possibly misaligned) 32-B piece: e[0..8] are the aligned dwords covering [q - s, q - s + 36).
struct RawPiece {
  uint32_t e[9];
};

__device__ __forceinline__ void issue_piece(RawPiece& r, const uint8_t* q, uint32_t s) {
  const u32x4a4* v = reinterpret_cast<const u32x4a4*>(q - s);
  const u32x4a4 x0 = v[0], x1 = v[1];
  r.e[0] = x0.x; r.e[1] = x0.y; r.e[2] = x0.z; r.e[3] = x0.w;
  r.e[4] = x1.x; r.e[5] = x1.y; r.e[6] = x1.z; r.e[7] = x1.w;
  // the 9th dword holds the piece's last byte(s) only when misaligned (never past the block);
  // aligned (s uniform 0) it re-reads the 8th, so the instruction is issued either way
  r.e[8] = *reinterpret_cast<const uint32_t*>(q - s + (s ? 32 : 28));
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
// kPack (kSync == 0 only): finished blocks are not folded one by one; each block's rotated lane
// partials are parked (up to 4 per wave, with their index and descriptor) and the 4 blocks are
// folded by ONE packed tree (tree4_packed: 7 shift operations per 4 blocks instead of 24), then
// lanes 0..3 hand block r's state to the sink.  A block with no 32-B piece parks its head state
// in lane 63 (the tree's unshifted position).
template <class Src, class Sink, int kSync, bool kDyn = false, bool kPack = false>
__global__ __launch_bounds__(kThreads) void crc_stream_kernel(const uint32_t* __restrict__ tabs,
                                                               Src src, uint64_t nblk, Sink sink) {
  static_assert(!kPack || kSync == 0, "packed trees need free-running waves");
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
  RawPiece na, nb, nc;
  uint32_t nhw = 0, nhb = 0;
  // Unmasked, unconditional loads (as in crc_stream16_kernel): a lane past the block's last
  // piece re-reads it, a lane with no head word reads the table buffer; a masked load would make
  // the next item's loads wait for this item's.
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(tabs);
  auto issue = [&](const BlkDesc& bd, uint32_t kk) {
    const uint32_t t = bd.n & 31u, K = bd.n >> 5;
    const uint8_t* q0 = K ? bd.p + t : dummy;
    const uint32_t s = K ? static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
                               static_cast<uint32_t>(reinterpret_cast<uintptr_t>(q0) & 3u)))
                         : 0u;
    const uint32_t cmax = K ? K - 1u : 0u;
    const uint32_t ca = u + (kk << 7), cb = ca + 64u, cc = ca + 128u;
    const bool last = kk + 1 >= rounds32(K);
    issue_piece(na, q0 + static_cast<uint64_t>(min(ca, cmax)) * 32u, s);
    issue_piece(nb, q0 + static_cast<uint64_t>(min(cb, cmax)) * 32u, s);
    issue_piece(nc, q0 + static_cast<uint64_t>(min(last ? cc : cb, cmax)) * 32u, s);  // chain c: last round
    const uint32_t lead = t & 3u, nh = t >> 2;
    const bool hw_on = kk == 0 && nh, hb_on = kk == 0 && lead;
    const uint32_t hs = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(reinterpret_cast<uintptr_t>(bd.p + lead) & 3u)));
    const uint8_t* hp = hw_on ? bd.p + lead + 4u * (min(max(u, 1u), nh) - 1u) - hs : dummy;
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(hp);
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(hp + (hw_on && hs ? 4u : 0u));
    nhw = __builtin_amdgcn_alignbyte(w1, w0, hw_on ? hs : 0u);
    const uint8_t* bp = hb_on ? bd.p : dummy;
    const uint32_t lm = hb_on ? lead - 1u : 0u;
    const uint32_t b0 = bp[0], b1 = bp[min(1u, lm)], b2 = bp[min(2u, lm)];
    nhb = b0 | (lead > 1 ? b1 << 8 : 0u) | (lead > 2 ? b2 << 16 : 0u);
  };
  if (active) {
    d = src.get(i);
    issue(d, 0);
  }
  // descriptor lookahead: the block after the one being loaded, its descriptor load in flight
  // (a descriptor fetched only when its block is due would put one full memory latency in front
  // of every block's loads)
  uint64_t ia = active ? next_block(i) : nend;
  typename Src::Raw ra = src.load(ia < nend ? ia : (nend ? nend - 1 : 0));
  uint32_t acc = 0;
  // kPack: parked blocks
  uint32_t park0 = 0, park1 = 0, park2 = 0, park3 = 0, npark = 0;
  uint64_t pid0 = 0, pid1 = 0, pid2 = 0, pid3 = 0;
  BlkDesc pd0{}, pd1{}, pd2{}, pd3{};
  auto flush = [&]() {
    const uint32_t v = tree4_packed<kDyn>(lds, u, park0, park1, park2, park3);
    if (u < npark) {
      const uint64_t id = u == 0 ? pid0 : (u == 1 ? pid1 : (u == 2 ? pid2 : pid3));
      const BlkDesc bd = u == 0 ? pd0 : (u == 1 ? pd1 : (u == 2 ? pd2 : pd3));
      sink.put(id, v, bd);
    }
    npark = 0;
    park0 = park1 = park2 = park3 = 0;
  };
  // kSync (equal lengths): every wave of the workgroup runs as many items as its first wave
  // (the one with the most blocks), so a plain barrier per item needs no LDS reduction.
  uint64_t items_left = 0, item = 0;
  if constexpr (kSync > 0) {
    const uint64_t wg_first = static_cast<uint64_t>(blockIdx.x) * kWavesPerWg;
    if (wg_first >= nblk) return;
    const uint32_t n0 = src.get(wg_first).n, K0 = n0 >> 5;
    items_left = ((nblk - wg_first + nw - 1) / nw) * rounds32(K0);
  }
  for (;;) {
    if constexpr (kSync > 0) {
      if (items_left-- == 0) break;
      if ((item++ % kSync) == 0) __syncthreads();
      if (!active) continue;
    }
    const RawPiece ca_ = na, cb_ = nb, cc_ = nc;
    const uint32_t chw = nhw, chb = nhb;
    const BlkDesc cd = d;
    const uint32_t ck = k;
    const uint32_t K = cd.n >> 5;
    const uint32_t R = rounds32(K);
    const bool last_round = ck + 1 >= R;
    const uint64_t ni = last_round ? ia : i;
    const bool have_next = ni < nend;
    if (last_round && have_next) {
      d = src.finish(ra);
      ia = next_block(ni);
    }
    // unconditional loads (see issue): the lookahead descriptor (clamped) and the next item (an
    // exhausted wave re-reads round 0 of its last block)
    ra = src.load(ia < nend ? ia : nend - 1);
    k = last_round ? 0 : ck + 1;
    issue(d, k);

    if (ck == 0) {  // head: every lane hashes the same (broadcast) head bytes from the seed
      const uint32_t t = cd.n & 31u, lead = t & 3u, nh = t >> 2;
      uint32_t h = cd.init_raw;
      const uint32_t lb = __builtin_amdgcn_readfirstlane(chb);
      if (lead) h = stepk(lds, lt, h, lb, lead);  // the 1-3 leading bytes in one table step
      for (uint32_t j = 0; j < nh; ++j) h = step4(lds, lt, h, __builtin_amdgcn_readlane(chw, j + 1));
      acc = (u == 0) ? h : 0u;
    }
    const uint32_t s = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(cd.p + (cd.n & 31u)) & 3u);
    const uint32_t ca = u + (ck << 7), cb = ca + 64u, cc = ca + 128u;
    // Every chain the round needs runs once for the whole wave (wave-uniform conditions: is there
    // any lane with a second / third piece?) and lanes without that piece discard it by select:
    // per-lane if/else would serialise the 1-, 2- and 3-chain cases of a partial round.
    {
      const uint32_t c0 = ck << 7;
      const bool anyb = K > c0 + 64u, anyc = last_round && K > c0 + 128u;  // wave-uniform
      const uint32_t start = ck ? shift_op(lds, PDB_SLOT_HORNER, acc) : acc;
      const uint32_t xa = chain_piece(lds, lt, start, ca_, s);
      uint32_t xb = 0, xc = 0;
      if (anyb) xb = chain_piece(lds, lt, 0u, cb_, s);
      if (anyc) xc = chain_piece(lds, lt, 0u, cc_, s);
      uint32_t v = ca < K ? xa : acc;  // a lane with no piece this round keeps its partial
      if (anyb) {
        const uint32_t vb = shift_op_x(lds, 7, xa, xb);
        v = cb < K ? vb : v;
      }
      if (anyc) {
        const uint32_t vc = shift_op_x(lds, 7, v, xc);
        v = (cc < K) ? vc : v;
      }
      acc = v;
    }
    if (last_round) {
      if constexpr (kPack) {
        uint32_t part;
        if (K) {
          const uint32_t q = K & 63u;
          part = q ? __shfl(acc, (u + q) & 63u, 64) : acc;
        } else {
          part = __builtin_amdgcn_readfirstlane(acc);  // head state (lane 0)
          part = u == 63u ? part : 0u;
        }
        switch (npark) {  // wave-uniform
          case 0: park0 = part; pid0 = i; pd0 = cd; break;
          case 1: park1 = part; pid1 = i; pd1 = cd; break;
          case 2: park2 = part; pid2 = i; pd2 = cd; break;
          default: park3 = part; pid3 = i; pd3 = cd; break;
        }
        if (++npark == 4) flush();
      } else {
        uint32_t raw = acc;
        if (K) {
          const uint32_t q = K & 63u;
          if (q) acc = __shfl(acc, (u + q) & 63u, 64);
          raw = wave_tree_dpp<kDyn>(lds, u, acc);
        }
        if (u == 0) sink.put(i, raw, cd);
      }
      i = ni;
      if (!have_next) {
        active = false;
        if constexpr (kSync == 0) break;
      }
    }
  }
  if constexpr (kPack) {
    if (npark) flush();
  }
}

// ---- coalesced stream kernel: 16-B lane pieces, every load instruction 1 KiB contiguous ------
// Same scheduling as crc_stream_kernel (one wave per block, items = 4-KiB rounds prefetched one
// ahead, workgroup-local dynamic blocks), with the load shape the nt calibration favours:
//   block of n bytes = head (t = n % 16 bytes) + K = n / 16 pieces of 16 B at q0 = p + t + 16c;
//   round r holds pieces c = 256r + 64j + u (j = 0..3) -> lane u, chain j, so load instruction j
//   of a round reads 1 KiB contiguous.  A lane's 4 chains (4 words each) fold as
//   a = x0, a = shift1024(a) ^ xj (slot 7); rounds chain with start = shift1008(acc) (slot 6)
//   injected into chain 0; rotation by K % 64 and the 6-level tree with slots 0..5 = 16 << k.
// Misaligned q0 (s = q0 & 3): each lane loads the 4-B aligned 16 B at q0 + 16c - s and takes
// the 17th..20th byte -- the next lane's first dword -- by DPP wave_shl:1 (lane 63: lane 0 of
// the next chain by readlane); only the lane ending a round's last chain or the block's last
// piece loads that dword itself.
template <bool kNT>
__device__ __forceinline__ u32x4 ldq(const uint8_t* q) {
  const u32x4a4* v = reinterpret_cast<const u32x4a4*>(q);
  if constexpr (kNT)
    return __builtin_nontemporal_load(v);
  else
    return *v;
}

template <class LT>
__device__ __forceinline__ uint32_t chain16(const char* lds, const LT& lt, uint32_t start,
                                            const u32x4& e, uint32_t nx, uint32_t s) {
  uint32_t w0 = e.x, w1 = e.y, w2 = e.z, w3 = e.w;
  if (s) {
    w0 = __builtin_amdgcn_alignbyte(e.y, e.x, s);
    w1 = __builtin_amdgcn_alignbyte(e.z, e.y, s);
    w2 = __builtin_amdgcn_alignbyte(e.w, e.z, s);
    w3 = __builtin_amdgcn_alignbyte(nx, e.w, s);
  }
  uint32_t x = start ^ w0;
  x = step4x(lds, lt, x, w1);
  x = step4x(lds, lt, x, w2);
  x = step4x(lds, lt, x, w3);
  return step4x(lds, lt, x, 0u);
}

// chain16 with its last word still unshifted (the final table step deferred to after the folds,
// as in partial4k_q)
template <class LT>
__device__ __forceinline__ uint32_t chain16p(const char* lds, const LT& lt, uint32_t start, const u32x4& e, uint32_t nx,
                                             uint32_t s) {
  uint32_t w0 = e.x, w1 = e.y, w2 = e.z, w3 = e.w;
  if (s) {
    w0 = __builtin_amdgcn_alignbyte(e.y, e.x, s);
    w1 = __builtin_amdgcn_alignbyte(e.z, e.y, s);
    w2 = __builtin_amdgcn_alignbyte(e.w, e.z, s);
    w3 = __builtin_amdgcn_alignbyte(nx, e.w, s);
  }
  uint32_t x = start ^ w0;
  x = step4x(lds, lt, x, w1);
  x = step4x(lds, lt, x, w2);
  return step4x(lds, lt, x, w3);
}

// LT: the table image -- QuadTabs (lane-quarter: T0..T3, shift 1024 and shift 1008 conflict-free;
// shipped) or LaneTabs (32 replicas of T0..T3, single-copy operators; A/B diagnostics).
// kBal (descriptor lists): byte-balanced workgroup ranges (bal_bound) instead of equal block counts.
// kDeferF: every chain stops with its last word unshifted (chain16p); the lane accumulator is
// finished by ONE table step where a round hands it on (before shift 1008) and after the final
// tree, instead of one step per chain (false: round 2 -- A/B).
// kLoadsOnly (diagnostics: the C3 row's pattern ceiling, bench.py): the same scheduling, descriptor
// lookahead and load instructions with NO hash -- every loaded word XOR-ed into the lane's
// accumulator, lane 0's written per block (wrong CRCs by design).
template <class Src, class Sink, bool kDyn, bool kNT, bool kPack = false, class LT = QuadTabs, bool kBal = false,
          bool kDeferF = true, bool kLoadsOnly = false>
__global__ __launch_bounds__(kThreads) void crc_stream16_kernel(const uint32_t* __restrict__ tabs,
                                                                 Src src, uint64_t nblk, Sink sink) {
  constexpr bool kQuad = __is_same(LT, QuadTabs);
  // the 32-replica image leaves no free slot: its work counter takes slot 5 (the trees then apply
  // shift 256 twice); the lane-quarter image leaves slots 6 and 7 free
  constexpr bool kL5Twice = kDyn && !kQuad;
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  if constexpr (kQuad)
    stage_tables_q4<PDB_CAT_TREE16, PDB_CAT_H1008, PDB_CAT_TREE16>(lds, tabs);  // image 1 hi: tree level 0
  else
    stage_tables<PDB_CAT_TREE16, PDB_CAT_H1008, PDB_CAT_S1024, kDyn>(lds, tabs);
  uint32_t* ctr = reinterpret_cast<uint32_t*>(lds + PDB_MAIN_BYTES + (kQuad ? 7u : 5u) * 4096u);
  uint64_t g_lo = nblk * blockIdx.x / gridDim.x, g_hi = nblk * (blockIdx.x + 1) / gridDim.x;
  static_assert(!kBal || (kDyn && kQuad), "byte balance: dynamic scheduling, lane-quarter image (slot 7)");
  uint64_t* bnd = reinterpret_cast<uint64_t*>(ctr + 2);  // kBal: this workgroup's range, from wave 0
  if constexpr (kBal) {
    if (threadIdx.x < 64) {
      const uint64_t lo = bal_bound(src, nblk, blockIdx.x, gridDim.x, threadIdx.x);
      const uint64_t hi = bal_bound(src, nblk, blockIdx.x + 1, gridDim.x, threadIdx.x);
      if (threadIdx.x == 0) bnd[0] = lo, bnd[1] = hi;
    }
  }
  if (kDyn && threadIdx.x == 0) *ctr = kWavesPerWg;  // next block, relative to g_lo
  __syncthreads();
  if constexpr (kBal) g_lo = bnd[0], g_hi = bnd[1];
  const uint32_t u = threadIdx.x & 63u;
  LT lt;
  if constexpr (kQuad)
    lt = quad_tabs(u);
  else
    lt = lane_tabs(u);
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
  if (i >= nend) return;

  // item = (block descriptor, block index, round); its loads live in a Buf16
  struct Meta {
    BlkDesc d;
    uint64_t i;
    uint32_t k;
    bool v;
  };
  struct Buf16 {
    u32x4 e[5];
    uint32_t nxt, hw, hb;
  };
  // Every item issues the same load instructions with every lane active and no branch around
  // any of them: a lane with nothing to load re-reads a valid address (the block's last piece, or
  // the table buffer `tabs` as a dummy), and the values it gets are never used.  A masked load
  // keeps its register's old value in inactive lanes, which makes the compiler wait for the
  // previous item's loads before issuing the next ones (no prefetch at all); a branch around a
  // load makes its vmcnt bookkeeping conservative.  Fixed, unmasked loads keep hashing an item
  // waiting only for that item's data.
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(tabs);
  auto issue = [&](Buf16& b, const BlkDesc& bd, uint32_t kk) {
    const uint32_t t = bd.n & 15u, K = bd.n >> 4;
    const uint8_t* q0 = bd.p + t;
    const uint32_t s = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(reinterpret_cast<uintptr_t>(q0) & 3u)));
    const uint8_t* qa = K ? q0 - s : dummy;
    const uint32_t cmax = K ? K - 1u : 0u;
    const uint32_t c0 = kk << 8;
    const bool last = kk + 1 >= rounds16(K);  // wave-uniform
#pragma unroll
    for (int j = 0; j < 4; ++j) b.e[j] = ldq<kNT>(qa + 16ull * min(c0 + 64u * j + u, cmax));
    // chain 4 exists only in the last round; otherwise re-read chain 3's (cached) piece
    b.e[4] = ldq<kNT>(qa + 16ull * min(c0 + (last ? 256u : 192u) + u, cmax));
    // the dword after a piece whose right neighbour is not in this round's registers: lane 63's
    // chain-3 piece in a non-last round (its neighbour opens the next round), and the block's
    // last piece (always in the last round); with s == 0 nothing is needed (re-read inside)
    const uint32_t cx = (u == 63u && !last) ? c0 + 255u : cmax;
    b.nxt = *reinterpret_cast<const uint32_t*>(qa + 16ull * cx + (s ? 16u : 0u));
    // head (round 0): word j (unaligned, hs) on lane j + 1, lead bytes on every lane
    const uint32_t lead = t & 3u, nh = t >> 2;
    const bool hw_on = kk == 0 && nh, hb_on = kk == 0 && lead;
    const uint32_t hs = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(reinterpret_cast<uintptr_t>(bd.p + lead) & 3u)));
    const uint8_t* hp = hw_on ? bd.p + lead + 4u * (min(max(u, 1u), nh) - 1u) - hs : dummy;
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(hp);
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(hp + (hw_on && hs ? 4u : 0u));
    b.hw = __builtin_amdgcn_alignbyte(w1, w0, hs);
    const uint8_t* bp = hb_on ? bd.p : dummy;
    const uint32_t lm = hb_on ? lead - 1u : 0u;
    const uint32_t b0 = bp[0], b1 = bp[min(1u, lm)], b2 = bp[min(2u, lm)];
    b.hb = b0 | (lead > 1 ? b1 << 8 : 0u) | (lead > 2 ? b2 << 16 : 0u);
  };

  // descriptor lookahead: block ia's descriptor is loaded one block before it is due.  Every
  // iteration issues exactly one descriptor load and one item's loads, whatever the block
  // geometry (an exhausted wave re-loads its last item as a dummy): a data-dependent branch
  // around a load makes the compiler's vmcnt bookkeeping conservative, and the wait for the
  // current item would then also wait for the loads just issued for the next one.
  uint64_t ia = next_block(i);
  typename Src::Raw ra = src.load(ia < nend ? ia : nend - 1);
  auto advance = [&](const Meta& m) -> Meta {  // the item after m (m.d is always a real block)
    Meta r{m.d, m.i, m.k, false};
    if (m.v && m.k + 1 < rounds16(m.d.n >> 4)) {
      r = Meta{m.d, m.i, m.k + 1, true};
    } else if (m.v && ia < nend) {
      r = Meta{src.finish(ra), ia, 0, true};
      ia = next_block(ia);
      // a block past 64 KiB goes to the long-block lane, and the wave takes the one after it (rare:
      // that descriptor is loaded when needed)
      while (src.long_export(r.i, r.d, u, kLongMinStream)) {
        if (ia >= nend) {
          r.v = false;
          break;
        }
        r = Meta{src.get(ia), ia, 0, true};
        ia = next_block(ia);
      }
    }
    ra = src.load(ia < nend ? ia : nend - 1);
    return r;
  };
  Meta mB{src.get(i), i, 0, true};
  while (src.long_export(mB.i, mB.d, u, kLongMinStream)) {  // (the wave's first block)
    if (ia >= nend) {
      mB.v = false;
      break;
    }
    mB = Meta{src.finish(ra), ia, 0, true};
    ia = next_block(ia);
    ra = src.load(ia < nend ? ia : nend - 1);
  }
  Buf16 B{};
  issue(B, mB.d, 0);
  uint32_t acc = 0;
  uint32_t park0 = 0, park1 = 0, park2 = 0, park3 = 0, npark = 0;
  uint32_t pfin = 0;  // kDeferF: bit r = parked block r is a head-only block (its part is a full state)
  uint64_t pid0 = 0, pid1 = 0, pid2 = 0, pid3 = 0;
  BlkDesc pd0{}, pd1{}, pd2{}, pd3{};
  auto flush = [&]() {
    uint32_t v;
    if constexpr (kQuad)
      v = tree4_packed<kL5Twice>(lds, u, park0, park1, park2, park3, QuadTree<128, -1>{lt});
    else
      v = tree4_packed<kL5Twice>(lds, u, park0, park1, park2, park3);
    if constexpr (kDeferF) {  // F: the chains' last words (lane r holds block r)
      const uint32_t f = step4x(lds, lt, v, 0u);
      v = ((pfin >> (u & 3u)) & 1u) ? v : f;
      pfin = 0;
    }
    if (u < npark) {
      const uint64_t id = u == 0 ? pid0 : (u == 1 ? pid1 : (u == 2 ? pid2 : pid3));
      const BlkDesc bd = u == 0 ? pd0 : (u == 1 ? pd1 : (u == 2 ? pd2 : pd3));
      sink.put(id, v, bd);
    }
    npark = 0;
    park0 = park1 = park2 = park3 = 0;
  };
  for (;;) {
    const Buf16 cur = B;
    const Meta mcur = mB;
    if (!mcur.v) break;
    mB = advance(mcur);
    issue(B, mB.d, mB.k);  // unconditional (see above)
    const u32x4 e0 = cur.e[0], e1 = cur.e[1], e2 = cur.e[2], e3 = cur.e[3], e4 = cur.e[4];
    const uint32_t cx = cur.nxt, chw = cur.hw, chb = cur.hb;
    const BlkDesc cd = mcur.d;
    const uint32_t ck = mcur.k;
    const uint32_t K = cd.n >> 4;
    const bool last_round = ck + 1 >= rounds16(K);
    if constexpr (kLoadsOnly) {
      const u32x4 x = (e0 ^ e1) ^ (e2 ^ e3) ^ e4;
      acc ^= xor3(xor3(x.x, x.y, x.z), x.w, xor3(cx, chw, chb));
      if (last_round && u == 0) sink.put(mcur.i, acc, cd);
      continue;
    }

    if (ck == 0) {  // head: every lane hashes the same (broadcast) head bytes from the seed
      const uint32_t t = cd.n & 15u, lead = t & 3u, nh = t >> 2;
      uint32_t h = cd.init_raw;
      const uint32_t lb = __builtin_amdgcn_readfirstlane(chb);
      if (lead) h = stepk(lds, lt, h, lb, lead);  // the 1-3 leading bytes in one table step
      for (uint32_t j = 0; j < nh; ++j) h = step4(lds, lt, h, __builtin_amdgcn_readlane(chw, j + 1));
      acc = (u == 0) ? h : 0u;
    }
    const uint32_t c0 = ck << 8;
    const uint32_t rem = K - c0;  // pieces left from this round on (>= 1 unless K == 0)
    // chains this lane runs: 4 in a full round; the last round holds up to 256 + 64 pieces
    const uint32_t J = !last_round ? 4u : (rem > u ? ((rem - u - 1u) >> 6) + 1u : 0u);
    // neighbour dwords for misaligned pieces, computed with every lane active (DPP sources)
    const uint32_t s = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(cd.p + (cd.n & 15u)) & 3u);
    uint32_t n0 = 0, n1 = 0, n2 = 0, n3 = 0, n4 = 0;
    if (s) {  // uniform branch
      // lane u+1's first dword (wave_shl:1); lane 63 keeps `old` = lane 0 of the next chain, or
      // for chain 3 of a non-last round the dword it loaded itself
      const bool five = last_round && rem > 256u;  // a fifth chain holds piece c0 + 256
      n0 = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(e1.x, 0), e0.x, 0x130, 0xF, 0xF, false);
      n1 = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(e2.x, 0), e1.x, 0x130, 0xF, 0xF, false);
      n2 = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(e3.x, 0), e2.x, 0x130, 0xF, 0xF, false);
      n3 = __builtin_amdgcn_update_dpp(five ? __builtin_amdgcn_readlane(e4.x, 0) : cx, e3.x, 0x130, 0xF, 0xF, false);
      n4 = __builtin_amdgcn_update_dpp(cx, e4.x, 0x130, 0xF, 0xF, false);
      // the block's last piece takes the dword its lane loaded itself
      const uint32_t cl = K - 1u;
      if (K && last_round && (cl & 63u) == u) {
        const uint32_t jl = (cl - c0) >> 6;
        n0 = jl == 0 ? cx : n0;
        n1 = jl == 1 ? cx : n1;
        n2 = jl == 2 ? cx : n2;
        n3 = jl == 3 ? cx : n3;
        n4 = jl == 4 ? cx : n4;
      }
    }
    if (J) {
      // chain j runs (once, for the whole wave) only if some lane has a piece in it: a block of
      // 1 KiB needs 2 of the 5 chains, not all of them (wave-uniform conditions on rem)
      // (kDeferF: the accumulator of the rounds before is finished first)
      const uint32_t start = ck ? round1008(lds, lt, kDeferF ? step4x(lds, lt, acc, 0u) : acc) : acc;
      const bool full = !last_round;
      auto ch = [&](uint32_t st0, const u32x4& e, uint32_t nx) {
        return kDeferF ? chain16p(lds, lt, st0, e, nx, s) : chain16(lds, lt, st0, e, nx, s);
      };
      uint32_t a = ch(start, e0, n0);
      // shift 1024: slot 7 of the 32-replica image (its slot 6 holds 1008), image 0 of the other
      auto fold = [&](uint32_t x, uint32_t y) {
        if constexpr (kQuad)
          return horner1024(lds, lt, x, y);
        else
          return shift_op_x(lds, 7, x, y);
      };
      if (full || rem > 64u) {
        const uint32_t x1 = ch(0u, e1, n1);
        if (J > 1) a = fold(a, x1);
      }
      if (full || rem > 128u) {
        const uint32_t x2 = ch(0u, e2, n2);
        if (J > 2) a = fold(a, x2);
      }
      if (full || rem > 192u) {
        const uint32_t x3 = ch(0u, e3, n3);
        if (J > 3) a = fold(a, x3);
      }
      if (!full && rem > 256u) {  // the last round's fifth chain
        const uint32_t x4 = ch(0u, e4, n4);
        if (J > 4) a = fold(a, x4);
      }
      acc = a;
    }
    if (last_round) {
      if constexpr (kPack) {
        uint32_t part;
        if (K) {
          const uint32_t q = K & 63u;
          part = q ? __shfl(acc, (u + q) & 63u, 64) : acc;
        } else {
          part = __builtin_amdgcn_readfirstlane(acc);  // head state (lane 0)
          part = u == 63u ? part : 0u;
        }
        if (kDeferF && !K) pfin |= 1u << npark;  // wave-uniform
        switch (npark) {  // wave-uniform
          case 0: park0 = part; pid0 = mcur.i; pd0 = cd; break;
          case 1: park1 = part; pid1 = mcur.i; pd1 = cd; break;
          case 2: park2 = part; pid2 = mcur.i; pd2 = cd; break;
          default: park3 = part; pid3 = mcur.i; pd3 = cd; break;
        }
        if (++npark == 4) flush();
      } else {
        uint32_t raw = acc;
        if (K) {
          const uint32_t q = K & 63u;
          if (q) acc = __shfl(acc, (u + q) & 63u, 64);
          raw = wave_tree_dpp<kL5Twice>(lds, u, acc);
          if constexpr (kDeferF) raw = step4x(lds, lt, raw, 0u);
        }
        if (u == 0) sink.put(mcur.i, raw, cd);
      }
    }
  }
  if constexpr (kPack) {
    if (npark) flush();
  }
}

// ---- sstable-sized blocks: one exact 4-KiB body + a batched prefix ------------------------------
// Every data block TableBuilder emits is a little over block_size = 4096 B (table_builder.cc:
// 127-130; the CRC covers contents || type, 197-198): db_bench's are 4167-4175 B.  The generic
// stream kernels pay for that shape with a fifth chain (4 extra 16-B pieces run by the whole
// wave), a serial broadcast head and a lane rotation per block.  Here a block of n bytes,
// 4096 <= n <= 4352, is split as
//   prefix = its first m = n - 4096 bytes,  body = its last 4096 bytes (at bs = p + m)
// and hashed from state 0 with the seed folded in up front:
//   * prefix: front-padded with z = (-m) mod 16 zero bytes to E = ceil(m/16) <= 16 pieces.
//     Hashing 0^z || prefix from U[z] = shift^-z(0xFFFFFFFF) gives exactly R(prefix) from
//     Value()'s seed (the z zeros carry U[z] to 0xFFFFFFFF).  The prefixes of a wave's 4 blocks
//     are hashed together: row r (lanes 16r..16r+15) takes block r, lane w the 16 B ending
//     16 (15 - w) bytes before bs (zero-masked below p; never loading a dword wholly below p),
//     and a 4-level DPP row tree (shift 16..128) leaves the prefix state P_r in lane 16r.
//   * body: exactly crc_pack4k_kernel<kNP = 4>'s geometry -- lane u owns the 16-B pieces at
//     bs + 16u + 1024j, every load instruction 1 KiB contiguous and non-temporal, chains folded
//     by Horner with "shift 1024" -- with P_r injected as lane 0's starting state.  bs has any
//     alignment: 4-B aligned dwordx4 loads, the 17th-20th byte from the next lane by DPP, one
//     extra dword for the block's last piece (as crc_stream16_kernel).
//   * the 4 blocks' lane partials fold in one tree4_packed (no rotation: the body is exactly 256
//     pieces); lanes 0..3 hand the raw states to the sink.
// Workgroup g owns blocks [g*N/G, (g+1)*N/G) and its waves take 4-block groups from an LDS
// counter (slot 7; the measured locality of crc_pack4k_dyn_kernel).  Loads run one block ahead
// (body) and one group ahead (descriptors, prefixes), every one unmasked and unconditional.
// Blocks outside [4096, 4352] (an index / metaindex / a table's last data block) are deferred
// and hashed after the loop by the slow path (below).
// crc_sst1k_kernel is the same design for ~1-KiB blocks (WAL physical records: type || fragment
// of a ~1-KiB write batch, db/log_writer.cc:111-121): body = the last 1 KiB (one chain per lane,
// one block per chain), 8-block groups whose prefixes are hashed in rows of 8 lanes (fast range
// [1024, 1152]) and folded by one tree8_packed, half a group's bodies in flight; kBlk = 4 (A/B)
// keeps rows of 16 lanes ([1024, 1280]) and 4-block trees.
// Valid only for Value()-seeded CRCs (init 0xFFFFFFFF): SstSrc always, FixedSrc / DescSrc without
// an Extend seed.
constexpr uint32_t kSstMin = 4096u, kSstMax = 4096u + 256u;

// The 16 bytes at A (any alignment) with the bytes below `lo` zeroed.  Never reads an aligned
// dword wholly below lo, nor -- A 4-B aligned -- the dword after the piece.
// Loads through integer addresses (the kernel computes block addresses as integers: readlane
// halves, selects against a dummy): cast to global-address-space pointers, or the compiler emits
// flat loads, whose lgkmcnt would make every LDS lookup wait for them too.
typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) const u32x4a4 g_u32x4;

__device__ __forceinline__ uint32_t gload32(uintptr_t a) { return *reinterpret_cast<g_u32*>(a); }

// 16 B at any byte address (one global_load_dwordx4: the runtime runs the shader in unaligned
// access mode); the A/B form of the body loads without the neighbour dword (variant 70)
typedef u32x4 u32x4a1 __attribute__((aligned(1)));
typedef __attribute__((address_space(1))) const u32x4a1 g_u32x4u;
template <bool kNT>
__device__ __forceinline__ u32x4 gload128u(uintptr_t a) {
  if constexpr (kNT)
    return __builtin_nontemporal_load(reinterpret_cast<g_u32x4u*>(a));
  else
    return *reinterpret_cast<g_u32x4u*>(a);
}
template <bool kNT>
__device__ __forceinline__ u32x4 gload128(uintptr_t a) {
  if constexpr (kNT)
    return __builtin_nontemporal_load(reinterpret_cast<g_u32x4*>(a));
  else
    return *reinterpret_cast<g_u32x4*>(a);
}

// A descriptor load whose last dword is never used (a handle's size_hi) leaves that register
// free for reuse, and reusing the destination of a load in flight waits for the load: keep the
// whole 16 B live until the descriptor is consumed.
__device__ __forceinline__ void keep_alive(const u32x4& r) { asm volatile("" ::"v"(r.w)); }
__device__ __forceinline__ void keep_alive(uint64_t) {}

struct MaskedPiece {
  uint32_t e[5];
  uint32_t s;   // A & 3
  int32_t zl;   // lo - A (bytes to zero, before clamping to [0, 16])
};

__device__ __forceinline__ void issue_masked(MaskedPiece& f, uintptr_t A, uintptr_t lo) {
  const uintptr_t l4 = lo & ~static_cast<uintptr_t>(3);
  const uint32_t s = static_cast<uint32_t>(A & 3u);
  const uintptr_t a0 = A - s;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    uintptr_t ad = a0 + 4u * (i < 4 ? static_cast<uint32_t>(i) : (s ? 4u : 3u));
    ad = ad < l4 ? l4 : ad;
    f.e[i] = gload32(ad);
  }
  f.s = s;
  const intptr_t zl = static_cast<intptr_t>(lo - A);
  f.zl = zl < -1 ? -1 : (zl > 16 ? 16 : static_cast<int32_t>(zl));
}

// The piece's raw state from `start` (0 for zero pieces: the masked bytes are zeros).
template <class LT>
__device__ __forceinline__ uint32_t hash_masked(const char* lds, const LT& lt, const MaskedPiece& f,
                                                uint32_t start) {
  const uint32_t z = f.zl < 0 ? 0u : static_cast<uint32_t>(f.zl);
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t v = __builtin_amdgcn_alignbyte(f.e[i + 1], f.e[i], f.s);
    const uint32_t sh = z > 4u * i ? min(z - 4u * i, 4u) : 0u;
    w[i] = sh >= 4u ? 0u : (v & (0xFFFFFFFFu << (8u * sh)));
  }
  return chain16(lds, lt, start, u32x4{w[0], w[1], w[2], w[3]}, 0u, 0u);
}

// Start state of a masked piece: U[z] on the piece holding the block's first byte (0 <= lo - A <
// 16), else 0.  ureg: lane l holds U[l & 15].  All lanes must be active (bpermute).
__device__ __forceinline__ uint32_t masked_start(const MaskedPiece& f, uint32_t ureg) {
  const uint32_t z = static_cast<uint32_t>(f.zl) & 15u;
  const uint32_t uz = __shfl(ureg, z, 64);
  return (f.zl >= 0 && f.zl < 16) ? uz : 0u;
}

// Levels of the wave tree inside each row of 16 lanes, folded toward the row's LAST lane
// (row_shr never crosses a row): lane 16r + 15 gets sum_w shift(c_w, 16 (15 - w)).  A prefix of
// E pieces sits in the row's last E lanes, so L = ceil(log2 E) levels suffice (wave-uniform).
template <class TO = SlotTree>
__device__ __forceinline__ uint32_t row_suffix_tree(const char* lds, uint32_t lane, uint32_t c, uint32_t L,
                                                    const TO& to = TO{}) {
  uint32_t y;
  if (L > 0) {
    y = __builtin_amdgcn_update_dpp(0u, c, 0x111, 0xF, 0xF, false);  // row_shr:1
    if ((lane & 1u) == 1u) c = to.op(lds, 0, y, c);
  }
  if (L > 1) {
    y = __builtin_amdgcn_update_dpp(0u, c, 0x112, 0xF, 0xF, false);  // row_shr:2
    if ((lane & 3u) == 3u) c = to.op(lds, 1, y, c);
  }
  if (L > 2) {
    y = __builtin_amdgcn_update_dpp(0u, c, 0x114, 0xF, 0xF, false);  // row_shr:4
    if ((lane & 7u) == 7u) c = shift_op_x(lds, 2, y, c);
  }
  if (L > 3) {
    y = __builtin_amdgcn_update_dpp(0u, c, 0x118, 0xF, 0xF, false);  // row_shr:8
    if ((lane & 15u) == 15u) c = shift_op_x(lds, 3, y, c);
  }
  return c;
}

// Slow path: the raw state of one block of any length (Value() seed) on the whole wave.  The
// block is front-padded with zeros to V = 4096 * ceil(n / 4096) bytes; lane u hashes the pieces at
// 16u + 1024k of the padded span (k = 0 .. V/1024 - 1) as one Horner sequence (shift 1024 between
// consecutive pieces: the body's lane-partial geometry), zero-masked below p with U[z] on the piece
// holding p; then the 6-level wave tree.  Rows (1-KiB steps) wholly below p are skipped (a 300-B
// WAL fragment costs one chain, not four).  Split in two so the drain can issue block k+1's first
// body while block k is hashed: slow_issue (loads of the first 4-KiB body) and slow_finish.
struct SlowFirst {
  MaskedPiece f[4];
};

__device__ __forceinline__ uintptr_t slow_vbs(uintptr_t p, uint32_t n) {
  const uint32_t nb = static_cast<uint32_t>((static_cast<uint64_t>(n) + 4095u) >> 12);
  return p + n - (static_cast<uintptr_t>(nb) << 12);
}

// An empty block reads nothing of its own: its (discarded) loads go to `dummy`.
__device__ __forceinline__ void slow_issue(SlowFirst& sf, uintptr_t p, uint32_t n, uint32_t u, uintptr_t dummy) {
  const uintptr_t lo = n ? p : dummy;
  const uintptr_t v = (n ? slow_vbs(p, n) : dummy) + 16u * u;
#pragma unroll
  for (int j = 0; j < 4; ++j) issue_masked(sf.f[j], v + 1024u * j, lo);
}

template <class LT>
__device__ __forceinline__ uint32_t slow_finish(const char* lds, const LT& lt, uint32_t u, uint32_t ureg,
                                                const SlowFirst& sf, uintptr_t p, uint32_t n) {
  if (n == 0) return 0xFFFFFFFFu;
  const uint32_t nb = static_cast<uint32_t>((static_cast<uint64_t>(n) + 4095u) >> 12);
  const uintptr_t vbs = slow_vbs(p, n);
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (vbs + 1024u * (j + 1) > p)  // wave-uniform: a row holding block bytes
      acc = horner1024(lds, lt, acc, hash_masked(lds, lt, sf.f[j], masked_start(sf.f[j], ureg)));
  if (nb > 1) {  // full bodies, the next one loading while one is hashed
    MaskedPiece f[4], g[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) issue_masked(f[j], vbs + 4096u + 16u * u + 1024u * j, p);
    for (uint32_t q = 1; q < nb; ++q) {
      const uint32_t qn = q + 1 < nb ? q + 1 : q;  // the last body re-reads itself (unconditional)
#pragma unroll
      for (int j = 0; j < 4; ++j) issue_masked(g[j], vbs + (static_cast<uintptr_t>(qn) << 12) + 16u * u + 1024u * j, p);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = horner1024(lds, lt, acc, hash_masked(lds, lt, f[j], 0u));
#pragma unroll
      for (int j = 0; j < 4; ++j) f[j] = g[j];
    }
  }
  return __builtin_amdgcn_readfirstlane(wave_tree_dpp(lds, u, acc));
}

// A wave defers the blocks outside the fast range to a list (lane k holds the k-th, relative to
// the workgroup's first block) and hashes them with the slow path after its fast loop, so the slow
// path's registers never compete with the pipeline's; a full list ends the fast loop, is drained,
// and the pipeline restarts at the group it stopped at.
constexpr uint32_t kSlowList = 64u;

// kRows = body size in KiB: 4 (crc_sst4k_kernel) or 1 (crc_sst1k_kernel).
// kBlk = blocks per group: 4 (rows of 16 lanes hash the prefixes: <= 256 B) or, for 1-KiB bodies,
// 8 (rows of 8 lanes: prefixes <= 128 B, one packed tree per 8 blocks).
// LT: the table image -- QuadTabs (lane-quarter, conflict-free shift 1024; shipped) or LaneTabs (the
// 32-replica image with single-copy operators; A/B diagnostics)
// kUA (A/B, variant 70): body pieces loaded at their exact byte addresses (unaligned dwordx4)
// instead of 4-B aligned + the DPP neighbour dword + v_alignbyte.
// kDeferF: the body chains stop with their last word unshifted and ONE table step follows the tree
// (chain16p; false = every chain finished before the folds, round 2 -- A/B).
template <class Src, class Sink, bool kNT, int kRows, bool kDiagNoFold = false, int kBlk = 4, class LT = QuadTabs,
          bool kUA = false, bool kDeferF = true, uint32_t kW = kWavesPerWg>
__device__ __forceinline__ void sized_kernel_body(const uint32_t* __restrict__ tabs, Src src, uint64_t nblk,
                                                  Sink sink) {
  static_assert(kRows == 0 || kRows == 1 || kRows == 4, "no body (records <= 256 B), 1-KiB or 4-KiB bodies");
  static_assert(kBlk == 4 || (kBlk == 8 && kRows >= 1), "4-block groups, or 8 with 1- or 4-KiB bodies");
  constexpr uint32_t kRowLanes = 64u / kBlk, kRowShift = kBlk == 4 ? 4u : 3u;
  // kRows = 0: the whole block is a "prefix" (1..16 kRowLanes bytes), hashed by its row alone
  constexpr uint32_t kBody = 1024u * kRows, kMin = kRows ? kBody : 1u, kMax = kBody + 16u * kRowLanes;
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  // lane-quarter image: T0..T3 and shift 1024 conflict-free, slots 0..5 = 16..512
  if constexpr (__is_same(LT, QuadTabs))
    stage_tables_q4<PDB_CAT_TREE16, PDB_CAT_TREE16, PDB_CAT_TREE16 + 1>(lds, tabs);  // image 1: tree levels 0, 1
  else
    stage_tables<PDB_CAT_TREE16, PDB_CAT_S1024>(lds, tabs);  // slots 0..5 = 16..512, 6 = 1024
  uint32_t* ctr = reinterpret_cast<uint32_t*>(lds + PDB_MAIN_BYTES + 7 * 4096u);
  const uint64_t g_lo = nblk * blockIdx.x / gridDim.x, g_hi = nblk * (blockIdx.x + 1) / gridDim.x;
  if (threadIdx.x == 0) *ctr = kW;  // next kBlk-block group, in groups relative to g_lo
  // OkRing (SinkRing<Sink>::kOn, the verify's ok bytes): the waves take groups out of order, so a
  // wave's own ok bytes are 4-B pieces scattered over the array (4.15 MB of partial-line writes per
  // 1 M blocks for 1.05 MB of flags).  Instead every block's byte goes to a ring of 16 lines of 128
  // blocks (one 128-B cache line of flags; 64-B lines still cost two write-backs of each 128-B line)
  // in operator slot 6 (free in this image), each line with a count of its blocks done and the line
  // that owns its slot; the wave whose count completes a line stores it as ONE 64-lane 2-byte store
  // (128 contiguous bytes) and hands the slot to line + 16.  A wave whose line's slot still holds line
  // - 16 waits for it (its blocks are all taken, by waves that never wait on a later line: no cycle).
  // A deferred (slow-path) block marks its byte 0xFF, which the line store skips: it is stored
  // directly when hashed.
  // (slot 6 is free only in the lane-quarter image: the 32-replica image keeps shift 1024 there)
  constexpr bool kOkRing = SinkRing<Sink>::kOn && kRows == 4 && kBlk == 4 && __is_same(LT, QuadTabs);
  uint8_t* ok_ring = reinterpret_cast<uint8_t*>(lds + PDB_MAIN_BYTES + 6 * 4096u);
  uint32_t* ok_cnt = reinterpret_cast<uint32_t*>(lds + PDB_MAIN_BYTES + 6 * 4096u + 2048u);
  uint32_t* ok_tag = reinterpret_cast<uint32_t*>(lds + PDB_MAIN_BYTES + 6 * 4096u + 2112u);
  if constexpr (kOkRing) {
    if (threadIdx.x < 16u) {  // relative lines 0..15 own slots 0..15
      ok_cnt[threadIdx.x] = 0;
      ok_tag[threadIdx.x] = threadIdx.x;
    }
  }
  const uint32_t u = threadIdx.x & 63u;
  const uint32_t ureg = tabs[PDB_UNSHIFT_OFF + (u & 15u)];
  __syncthreads();
  LT lt;
  if constexpr (__is_same(LT, QuadTabs))
    lt = quad_tabs(u);
  else
    lt = lane_tabs(u);
  // tree levels 0 and 1 from image 1's replicated copies (lane-quarter image), else the slots
  auto tops = [&]() {
    if constexpr (__is_same(LT, QuadTabs))
      return QuadTree<0, 128>{lt};
    else
      return SlotTree{};
  };
  uint64_t grp = g_lo + kBlk * static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
  if (grp >= g_hi) return;
  const uintptr_t dummy = reinterpret_cast<uintptr_t>(tabs);  // >= 4 KiB + 256 B of valid bytes
  auto next_group = [&]() -> uint64_t {
    uint32_t r = 0;
    if (u == 0) r = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return g_lo + kBlk * static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(r));
  };
  // lane u holds block (group + (u % kBlk))'s descriptor (clamped into the range: a group past
  // the end re-reads the last block, never used)
  auto lane_idx = [&](uint64_t gg) -> uint64_t {
    const uint64_t i = gg + (u & (kBlk - 1u));
    return i < g_hi ? i : g_hi - 1;
  };
  auto load_desc = [&](uint64_t gg) { return src.load(lane_idx(gg)); };
  struct Grp {
    BlkDesc ld;         // per lane: block (u % kBlk)
    uintptr_t p[kBlk];  // uniform
    uint32_t n[kBlk];
  };
  auto finish = [&](const typename Src::Raw& raw) -> Grp {
    keep_alive(raw);
    Grp G;
    G.ld = src.lane(raw);
    const uintptr_t lp = reinterpret_cast<uintptr_t>(G.ld.p);
    const uint32_t lo = static_cast<uint32_t>(lp), hi = static_cast<uint32_t>(static_cast<uint64_t>(lp) >> 32);
#pragma unroll
    for (int r = 0; r < kBlk; ++r) {
      G.p[r] = static_cast<uintptr_t>(uniform64(__builtin_amdgcn_readlane(lo, r), __builtin_amdgcn_readlane(hi, r)));
      G.n[r] = __builtin_amdgcn_readlane(G.ld.n, r);
    }
    return G;
  };
  auto fast = [](uint32_t n) { return n - kMin <= kMax - kMin; };
  // parked trailers (SinkPark): this lane's slot, written kRing groups after it was filled
  // (rings of more than 16 groups: kRing / 16 slots per lane, slot (g / 16) mod (kRing / 16))
  constexpr uint32_t kRing = SinkPark<Sink>::kRing;
  constexpr uint32_t kPkS = kRing > 16u ? kRing / 16u : 1u, kPkL = kRing > 16u ? 16u : (kRing ? kRing : 1u);
  static_assert(kRing == 0 || (kRows == 4 && kBlk == 4), "parking: the sstable-sized seal");
  uintptr_t pk_a[kPkS];
  uint32_t pk_m[kPkS], pk_n = 0;
  bool pk_ok[kPkS];
#pragma unroll
  for (uint32_t k = 0; k < kPkS; ++k) pk_a[k] = 0, pk_m[k] = 0, pk_ok[k] = false;
  auto park = [&](uint32_t v, const Grp& G, uint32_t fastbits, uint32_t nv) {
    const uint32_t r = u & 3u;  // lane u holds block r's descriptor already
    const uint32_t m = pdb_mask(~static_cast<uint32_t>(__shfl(v, r, 64)));
    const bool ok = r < nv && ((fastbits >> r) & 1u) && G.ld.init_raw != 0;
    const uint32_t sub = (pk_n / kPkL) % kPkS;  // uniform
#pragma unroll
    for (uint32_t k = 0; k < kPkS; ++k)
      if (k == sub && (u >> 2) == (pk_n % kPkL)) {
        if (pk_ok[k]) write_trailer_word(pk_a[k], pk_m[k]);
        pk_a[k] = reinterpret_cast<uintptr_t>(G.ld.p) + G.ld.n;
        pk_m[k] = m;
        pk_ok[k] = ok;
      }
    ++pk_n;
  };
  // the group's ok bytes into the ring (lane u < nv: block grp + u), then the lines they complete
  // stored (see OkRing above)
  auto ok_ring_put = [&](uint32_t v, const Grp& G, uint32_t fastbits, uint32_t nv, uint32_t stored) {
    if constexpr (kOkRing) {
      // 32-bit, relative to the range: block r = grp - g_lo + u, line Lr = (r + lo7) / 128 (lines
      // of the flag array's 128-B grid, lo7 = g_lo mod 128), tags hold relative lines
      const bool mine = u < nv;
      const uint32_t lo7 = static_cast<uint32_t>(g_lo) & 127u, nrel = static_cast<uint32_t>(g_hi - g_lo);
      const uint32_t r = static_cast<uint32_t>(grp - g_lo) + u, rl = r + lo7;
      const uint32_t L = rl >> 7, slot = L & 15u;
      uint8_t b = 0xFFu;  // deferred: stored by the slow path
      if (mine && ((fastbits >> u) & 1u)) b = SinkOps<Sink>::verdict(sink, v, G.ld, stored);
      // wait until every lane's slot belongs to its line
      while (__builtin_amdgcn_ballot_w64(mine && __hip_atomic_load(ok_tag + slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != L))
        __builtin_amdgcn_s_sleep(1);
      bool done = false;
      if (mine) {
        ok_ring[slot * 128u + (rl & 127u)] = b;
        const uint32_t lb = L << 7;  // (in rl units)
        const uint32_t want = min(nrel + lo7, lb + 128u) - max(lo7, lb);
        done = __hip_atomic_fetch_add(ok_cnt + slot, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) + 1u == want;
      }
      uint64_t fin = __builtin_amdgcn_ballot_w64(done);
      while (fin) {  // at most two lines: a group straddles at most one line boundary
        const uint32_t k = static_cast<uint32_t>(__builtin_ctzll(fin));
        fin &= fin - 1;
        const uint32_t Lc = __builtin_amdgcn_readlane(L, k), sc = Lc & 15u;
        // lane u: blocks 2u, 2u + 1 of the line (rl units; the range is [lo7, nrel + lo7))
        const uint32_t j = (Lc << 7) + 2u * u;
        const uint32_t pair = *reinterpret_cast<const uint16_t*>(ok_ring + sc * 128u + 2u * u);
        const bool v0 = j >= lo7 && j < nrel + lo7 && (pair & 0xFFu) != 0xFFu;
        const bool v1 = j + 1u >= lo7 && j + 1u < nrel + lo7 && (pair >> 8) != 0xFFu;
        uint8_t* dst = sink.ok + (g_lo - lo7) + j;
        if (sink.ok) {
          if (v0 && v1)
            *reinterpret_cast<uint16_t*>(dst) = static_cast<uint16_t>(pair);
          else if (v0)
            dst[0] = static_cast<uint8_t>(pair);
          else if (v1)
            dst[1] = static_cast<uint8_t>(pair >> 8);
        }
        if (u == 0) {
          ok_cnt[sc] = 0;
          __hip_atomic_store(ok_tag + sc, Lc + 16u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
  };
  auto body_at = [&](const Grp& G, int r) -> uintptr_t {
    return fast(G.n[r]) ? G.p[r] + G.n[r] - kBody : dummy;
  };
  // body loads of one block: kRows x 16 B per lane (4-B aligned) + the dword after the last piece
  auto issue_body = [&](u32x4* b, uint32_t& last, uintptr_t bs) {
    const uint32_t s = static_cast<uint32_t>(bs & 3u);
    const uintptr_t q = bs - s;
    if constexpr (kUA) {
#pragma unroll
      for (int j = 0; j < kRows; ++j) b[j] = gload128u<kNT>(bs + 16u * u + 1024u * j);
      last = 0;
      (void)q;
    } else {
#pragma unroll
      for (int j = 0; j < kRows; ++j) b[j] = gload128<kNT>(q + 16u * u + 1024u * j);
      last = gload32(q + (s ? kBody : kBody - 4u));
    }
  };
  // prefix loads of a group: row r (kRowLanes lanes) takes block r, lane w the 16 B at
  // bs - 16 kRowLanes + 16w
  auto issue_prefix = [&](MaskedPiece& f, const Grp& G) {
    const uint32_t row = u >> kRowShift, w = u & (kRowLanes - 1u);
    // block `row`'s descriptor from lane `row` (bpermute: no per-lane indexing of G.p / G.n)
    const uint64_t lp = reinterpret_cast<uintptr_t>(G.ld.p);
    const uint32_t plo = __shfl(static_cast<uint32_t>(lp), row, 64), phi = __shfl(static_cast<uint32_t>(lp >> 32), row, 64);
    const uintptr_t p = static_cast<uintptr_t>((static_cast<uint64_t>(phi) << 32) | plo);
    const uint32_t n = __shfl(G.ld.n, row, 64);
    const bool ok = fast(n);
    const uintptr_t A = ok ? p + n - kMax + 16u * w : dummy + 16u * w;
    issue_masked(f, A, ok ? p : dummy + 256u);  // a slow block's row: all masked
  };
  // the group's prefix states: P_r in the row's last lane (E_r = 0, n = kBody: the seed itself);
  // the row tree runs only the levels the longest prefix of the group needs
  auto prefix_states = [&](const MaskedPiece& pf, const Grp& G, uint32_t (&P)[kBlk]) {
    uint32_t emax = 0;
#pragma unroll
    for (int r = 0; r < kBlk; ++r) {
      const uint32_t e = fast(G.n[r]) ? (G.n[r] - kMin + 15u) >> 4 : 0u;
      emax = e > emax ? e : emax;
    }
    const uint32_t L = emax <= 1 ? 0u : (emax <= 2 ? 1u : (emax <= 4 ? 2u : (emax <= 8 ? 3u : 4u)));
    const uint32_t pref = row_suffix_tree(lds, u, hash_masked(lds, lt, pf, masked_start(pf, ureg)), L, tops());
#pragma unroll
    for (int r = 0; r < kBlk; ++r) {
      // a block of exactly kBody bytes has no prefix: its start state is the seed itself
      // (Value()'s, or a long-block piece's own: SrcSeeds)
      const uint32_t seed = SrcSeeds<Src>::kOn ? __builtin_amdgcn_readlane(G.ld.init_raw, r) : 0xFFFFFFFFu;
      P[r] = (kRows && G.n[r] == kMin) ? seed : __builtin_amdgcn_readlane(pref, kRowLanes * r + kRowLanes - 1);
    }
  };
  // one body's lane partial: chains j (16-B pieces at bs + 16u + 1024j) with the DPP neighbour
  // dword, Horner-folded with shift 1024, P injected as lane 0's start
  auto body_partial = [&](const u32x4* e, uint32_t cl, uint32_t s, uint32_t P) -> uint32_t {
    uint32_t nx[kRows ? kRows : 1];  // (kRows = 0 has no body: never called)
#pragma unroll
    for (int j = 0; j < kRows; ++j) nx[j] = 0;
    if (s) {  // neighbour dwords: lane u + 1's first dword; lane 63 the next chain's lane 0
#pragma unroll
      for (int j = 0; j < kRows; ++j)
        nx[j] = __builtin_amdgcn_update_dpp(j + 1 < kRows ? __builtin_amdgcn_readlane(e[j + 1 < kRows ? j + 1 : j].x, 0) : cl,
                                            e[j].x, 0x130, 0xF, 0xF, false);
    }
    uint32_t a = kDeferF ? chain16p(lds, lt, u == 0 ? P : 0u, e[0], nx[0], s) : chain16(lds, lt, u == 0 ? P : 0u, e[0], nx[0], s);
#pragma unroll
    for (int j = 1; j < kRows; ++j) {
      const uint32_t x = kDeferF ? chain16p(lds, lt, 0u, e[j], nx[j], s) : chain16(lds, lt, 0u, e[j], nx[j], s);
      // kDiagNoFold (A/B diagnostics only, WRONG CRCs): the Horner fold replaced by a XOR, to price
      // the shift-operator lookups
      a = kDiagNoFold ? (a ^ x) : horner1024(lds, lt, a, x);
    }
    return a;
  };

  uint32_t slow = 0, nslow = 0;  // deferred blocks (lane k: the k-th, minus g_lo)
  auto defer = [&](const Grp& G, uint32_t fastbits, uint32_t nv) {
    const uint32_t slowbits = ~fastbits & ((1u << nv) - 1u);
    if (slowbits) {
#pragma unroll
      for (int r = 0; r < kBlk; ++r)
        if ((slowbits >> r) & 1u) {
          slow = u == nslow ? static_cast<uint32_t>(grp + r - g_lo) : slow;
          ++nslow;
        }
    }
  };
  auto fast_bits = [&](const Grp& G) {
    uint32_t fb = 0;
#pragma unroll
    for (int r = 0; r < kBlk; ++r) fb |= fast(G.n[r]) ? 1u << r : 0u;
    return fb;
  };
  uint64_t ngrp = next_group();
  for (;;) {  // (re)start the pipeline at grp (ngrp already taken from the counter)
    typename Src::Raw nraw = load_desc(ngrp);
    Grp G = finish(load_desc(grp));
    uint32_t pre = SinkOps<Sink>::pre(sink, lane_idx(grp), G.ld);
    MaskedPiece pf;
    issue_prefix(pf, G);
    bool done = false;
    if constexpr (kRows == 4) {
      // bodies one block ahead; the next group's descriptors, prefixes and first body at block 3
      u32x4 buf[4];
      uint32_t blast;
      issue_body(buf, blast, body_at(G, 0));
      for (;;) {
        uint32_t P[kBlk];
        prefix_states(pf, G, P);
        // what the sink reads for this group (the verify's stored trailers), issued here and used
        // after the group's four bodies: one such register live, not this group's and the next's
        // (a second one spilled the 12-wave verify)
        if constexpr (kOkRing) pre = SinkOps<Sink>::pre(sink, lane_idx(grp), G.ld);
        Grp NG = G;
        uint32_t npre = pre;
        MaskedPiece npf = pf;
        uint64_t nngrp = ngrp;
        uint32_t part[kBlk];
        const uint32_t nv = static_cast<uint32_t>(g_hi - grp < kBlk ? g_hi - grp : kBlk);
        const uint32_t fastbits = fast_bits(G);
#pragma unroll
        for (int r = 0; r < kBlk; ++r) {
          const u32x4 e[4] = {buf[0], buf[1], buf[2], buf[3]};
          const uint32_t cl = blast;
          if (r < kBlk - 1) {
            issue_body(buf, blast, body_at(G, r + 1));
          } else {
            NG = finish(nraw);
            issue_body(buf, blast, body_at(NG, 0));
            issue_prefix(npf, NG);
            if constexpr (!kOkRing) npre = SinkOps<Sink>::pre(sink, lane_idx(ngrp), NG.ld);
            if (ngrp < g_hi) nngrp = next_group();
            nraw = load_desc(nngrp < g_hi ? nngrp : ngrp);
          }
          part[r] = 0;
          if ((fastbits >> r) & 1u)
            part[r] = body_partial(e, cl, kUA ? 0u : static_cast<uint32_t>((G.p[r] + G.n[r]) & 3u), P[r]);
        }
        uint32_t v;
        if constexpr (kBlk == 4)
          v = tree4_packed(lds, u, part[0], part[1], part[2], part[3], tops());
        else
          v = tree8_packed(lds, u, part, tops());
        if constexpr (kDeferF) v = step4x(lds, lt, v, 0u);  // F: the body chains' last words
        if constexpr (kRing != 0)
          park(v, G, fastbits, nv);
        else if constexpr (kOkRing)
          ok_ring_put(v, G, fastbits, nv, pre);
        else if (u < nv && ((fastbits >> u) & 1u))
          SinkOps<Sink>::put(sink, grp + u, v, G.ld, pre);
        defer(G, fastbits, nv);
        if (ngrp >= g_hi) {
          done = true;
          break;
        }
        grp = ngrp;
        ngrp = nngrp;
        G = NG;
        pre = npre;
        pf = npf;
        if (nslow > kSlowList - kBlk) break;  // no room for another group's slow blocks: drain first
      }
    } else if constexpr (kRows == 0) {
      // records <= 256 B: no body, no tree -- a row's suffix tree leaves the block's raw state in
      // the row's last lane.  The next group's descriptors and prefix loads are in flight while
      // one group hashes.
      for (;;) {
        const MaskedPiece cpf = pf;
        const Grp NG = finish(nraw);
        issue_prefix(pf, NG);
        const uint32_t npre = SinkOps<Sink>::pre(sink, lane_idx(ngrp), NG.ld);
        uint64_t nngrp = ngrp;
        if (ngrp < g_hi) nngrp = next_group();
        nraw = load_desc(nngrp < g_hi ? nngrp : ngrp);
        uint32_t emax = 0;
#pragma unroll
        for (int r = 0; r < kBlk; ++r) {
          const uint32_t e = fast(G.n[r]) ? (G.n[r] + 15u) >> 4 : 0u;
          emax = e > emax ? e : emax;
        }
        const uint32_t L = emax <= 1 ? 0u : (emax <= 2 ? 1u : (emax <= 4 ? 2u : (emax <= 8 ? 3u : 4u)));
        const uint32_t pref = row_suffix_tree(lds, u, hash_masked(lds, lt, cpf, masked_start(cpf, ureg)), L, tops());
        const uint32_t v = __shfl(pref, (u & (kBlk - 1u)) * kRowLanes + kRowLanes - 1u, 64);  // lane r: block r
        const uint32_t nv = static_cast<uint32_t>(g_hi - grp < kBlk ? g_hi - grp : kBlk);
        const uint32_t fastbits = fast_bits(G);
        if (u < nv && ((fastbits >> u) & 1u)) SinkOps<Sink>::put(sink, grp + u, v, G.ld, pre);
        defer(G, fastbits, nv);
        if (ngrp >= g_hi) {
          done = true;
          break;
        }
        grp = ngrp;
        ngrp = nngrp;
        G = NG;
        pre = npre;
        if (nslow > kSlowList - kBlk) break;  // drain first (pf already holds grp's prefixes)
      }
    } else if constexpr (kBlk == 4) {
      // 1-KiB bodies: the next group's 4 bodies, prefixes and descriptors issued at the top of a
      // group (4 KiB + 1 KiB in flight per wave while this group hashes)
      u32x4 b0, b1, b2, b3;
      uint32_t l0, l1, l2, l3;
      issue_body(&b0, l0, body_at(G, 0));
      issue_body(&b1, l1, body_at(G, 1));
      issue_body(&b2, l2, body_at(G, 2));
      issue_body(&b3, l3, body_at(G, 3));
      for (;;) {
        const u32x4 c0 = b0, c1 = b1, c2 = b2, c3 = b3;
        const uint32_t cl0 = l0, cl1 = l1, cl2 = l2, cl3 = l3;
        const MaskedPiece cpf = pf;
        const Grp NG = finish(nraw);
        issue_body(&b0, l0, body_at(NG, 0));
        issue_body(&b1, l1, body_at(NG, 1));
        issue_body(&b2, l2, body_at(NG, 2));
        issue_body(&b3, l3, body_at(NG, 3));
        issue_prefix(pf, NG);
        const uint32_t npre = SinkOps<Sink>::pre(sink, lane_idx(ngrp), NG.ld);
        uint64_t nngrp = ngrp;
        if (ngrp < g_hi) nngrp = next_group();
        nraw = load_desc(nngrp < g_hi ? nngrp : ngrp);
        uint32_t P[4];
        prefix_states(cpf, G, P);
        const uint32_t nv = static_cast<uint32_t>(g_hi - grp < 4 ? g_hi - grp : 4);
        const uint32_t fastbits = fast_bits(G);
        uint32_t part[4] = {0, 0, 0, 0};
        if (fastbits & 1u) part[0] = body_partial(&c0, cl0, static_cast<uint32_t>((G.p[0] + G.n[0]) & 3u), P[0]);
        if (fastbits & 2u) part[1] = body_partial(&c1, cl1, static_cast<uint32_t>((G.p[1] + G.n[1]) & 3u), P[1]);
        if (fastbits & 4u) part[2] = body_partial(&c2, cl2, static_cast<uint32_t>((G.p[2] + G.n[2]) & 3u), P[2]);
        if (fastbits & 8u) part[3] = body_partial(&c3, cl3, static_cast<uint32_t>((G.p[3] + G.n[3]) & 3u), P[3]);
        uint32_t v = tree4_packed(lds, u, part[0], part[1], part[2], part[3], tops());
        if constexpr (kDeferF) v = step4x(lds, lt, v, 0u);  // F: the body chains' last words
        if (u < nv && ((fastbits >> u) & 1u)) SinkOps<Sink>::put(sink, grp + u, v, G.ld, pre);
        defer(G, fastbits, nv);
        if (ngrp >= g_hi) {
          done = true;
          break;
        }
        grp = ngrp;
        ngrp = nngrp;
        G = NG;
        pre = npre;
        if (nslow > kSlowList - kBlk) break;  // drain first (pf already holds grp's prefixes)
      }
    } else {
      // 1-KiB bodies, 8-block groups: half a group's bodies in flight -- blocks 4..7 load while
      // 0..3 hash, the next group's 0..3 (with its prefixes and the lookahead descriptors) while
      // 4..7 hash -- and one tree8_packed per 8 blocks
      u32x4 b0, b1, b2, b3;
      uint32_t l0, l1, l2, l3;
      issue_body(&b0, l0, body_at(G, 0));
      issue_body(&b1, l1, body_at(G, 1));
      issue_body(&b2, l2, body_at(G, 2));
      issue_body(&b3, l3, body_at(G, 3));
      for (;;) {
        uint32_t P[8];
        uint32_t part[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const uint32_t nv = static_cast<uint32_t>(g_hi - grp < 8 ? g_hi - grp : 8);
        const uint32_t fastbits = fast_bits(G);
        {  // blocks 0..3 (loaded a half-group ago); blocks 4..7 start loading
          const u32x4 c0 = b0, c1 = b1, c2 = b2, c3 = b3;
          const uint32_t cl0 = l0, cl1 = l1, cl2 = l2, cl3 = l3;
          issue_body(&b0, l0, body_at(G, 4));
          issue_body(&b1, l1, body_at(G, 5));
          issue_body(&b2, l2, body_at(G, 6));
          issue_body(&b3, l3, body_at(G, 7));
          prefix_states(pf, G, P);
          if (fastbits & 1u) part[0] = body_partial(&c0, cl0, static_cast<uint32_t>((G.p[0] + G.n[0]) & 3u), P[0]);
          if (fastbits & 2u) part[1] = body_partial(&c1, cl1, static_cast<uint32_t>((G.p[1] + G.n[1]) & 3u), P[1]);
          if (fastbits & 4u) part[2] = body_partial(&c2, cl2, static_cast<uint32_t>((G.p[2] + G.n[2]) & 3u), P[2]);
          if (fastbits & 8u) part[3] = body_partial(&c3, cl3, static_cast<uint32_t>((G.p[3] + G.n[3]) & 3u), P[3]);
        }
        const u32x4 c4 = b0, c5 = b1, c6 = b2, c7 = b3;
        const uint32_t cl4 = l0, cl5 = l1, cl6 = l2, cl7 = l3;
        const Grp NG = finish(nraw);
        issue_body(&b0, l0, body_at(NG, 0));
        issue_body(&b1, l1, body_at(NG, 1));
        issue_body(&b2, l2, body_at(NG, 2));
        issue_body(&b3, l3, body_at(NG, 3));
        issue_prefix(pf, NG);
        const uint32_t npre = SinkOps<Sink>::pre(sink, lane_idx(ngrp), NG.ld);
        uint64_t nngrp = ngrp;
        if (ngrp < g_hi) nngrp = next_group();
        nraw = load_desc(nngrp < g_hi ? nngrp : ngrp);
        if (fastbits & 16u) part[4] = body_partial(&c4, cl4, static_cast<uint32_t>((G.p[4] + G.n[4]) & 3u), P[4]);
        if (fastbits & 32u) part[5] = body_partial(&c5, cl5, static_cast<uint32_t>((G.p[5] + G.n[5]) & 3u), P[5]);
        if (fastbits & 64u) part[6] = body_partial(&c6, cl6, static_cast<uint32_t>((G.p[6] + G.n[6]) & 3u), P[6]);
        if (fastbits & 128u) part[7] = body_partial(&c7, cl7, static_cast<uint32_t>((G.p[7] + G.n[7]) & 3u), P[7]);
        uint32_t v = tree8_packed(lds, u, part, tops());
        if constexpr (kDeferF) v = step4x(lds, lt, v, 0u);  // F: the body chains' last words
        if (u < nv && ((fastbits >> u) & 1u)) SinkOps<Sink>::put(sink, grp + u, v, G.ld, pre);
        defer(G, fastbits, nv);
        if (ngrp >= g_hi) {
          done = true;
          break;
        }
        grp = ngrp;
        ngrp = nngrp;
        G = NG;
        pre = npre;
        if (nslow > kSlowList - kBlk) break;  // drain first (pf already holds grp's prefixes)
      }
    }
    // drain the deferred blocks, block k+1's descriptor and first body loading while k hashes
    // (the pipeline's loads in flight are abandoned)
    if (nslow) {
      auto idx = [&](uint32_t k) { return g_lo + __builtin_amdgcn_readlane(slow, k < nslow ? k : nslow - 1); };
      struct Slow {
        BlkDesc d;
        uintptr_t p;
        uint32_t n, pre;
        uint64_t i;
        SlowFirst sf;
      };
      auto stage = [&](Slow& S, uint64_t i, const typename Src::Raw& raw) {
        keep_alive(raw);
        S.i = i;
        S.d = src.lane(raw);
        const uint64_t lp = reinterpret_cast<uintptr_t>(S.d.p);
        S.p = static_cast<uintptr_t>(uniform64(static_cast<uint32_t>(lp), static_cast<uint32_t>(lp >> 32)));
        S.n = __builtin_amdgcn_readfirstlane(S.d.n);
        S.pre = SinkOps<Sink>::pre(sink, i, S.d);
        slow_issue(S.sf, S.p, S.n, u, dummy);
      };
      Slow cur;
      stage(cur, idx(0), src.load(idx(0)));
      typename Src::Raw rn = src.load(idx(1));
      for (uint32_t k = 0; k < nslow; ++k) {
        Slow nxt;
        stage(nxt, idx(k + 1), rn);  // past the end: re-stages the last block (unconditional)
        rn = src.load(idx(k + 2));
        // a long block (index / filter: up to MiBs) goes to the long-block lane instead of this wave
        const BlkDesc ud{reinterpret_cast<const uint8_t*>(cur.p), cur.n,
                          static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(cur.d.init_raw))};
        if (!src.long_export_cold(cur.i, ud, u, kLongMinBytes)) {
          const uint32_t raw_state = slow_finish(lds, lt, u, ureg, cur.sf, cur.p, cur.n);
          if (u == 0) SinkOps<Sink>::put(sink, cur.i, raw_state, cur.d, cur.pre);
        }
        cur = nxt;
      }
      nslow = 0;
    }
    if (done) break;
  }
  if constexpr (kRing != 0) {
#pragma unroll
    for (uint32_t k = 0; k < kPkS; ++k)
      if (pk_ok[k]) write_trailer_word(pk_a[k], pk_m[k]);
  }
}

// kBlk = 8 (A/B): 8-block groups, prefixes <= 128 B in rows of 8 lanes, one tree8_packed.
// kW: waves per workgroup (16 = 1024 threads, 128 VGPRs a lane; A/B diagnostics 12 / 8 waves).
template <class Src, class Sink, bool kNT, int kBlk = 4, class LT = QuadTabs, bool kUA = false, bool kDeferF = true,
          uint32_t kW = kWavesPerWg>
__global__ __launch_bounds__(kW * 64) void crc_sst4k_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                            uint64_t nblk, Sink sink) {
  sized_kernel_body<Src, Sink, kNT, 4, false, kBlk, LT, kUA, kDeferF, kW>(tabs, src, nblk, sink);
}

// (the 1-KiB body has no Horner fold: both images measure the same, +0.8 % for the lane-quarter
// one -- diagnostics variant 42 is the 32-replica image)
template <class Src, class Sink, bool kNT, int kBlk = 8, class LT = QuadTabs>
__global__ __launch_bounds__(kThreads) void crc_sst1k_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                             uint64_t nblk, Sink sink) {
  sized_kernel_body<Src, Sink, kNT, 1, false, kBlk, LT>(tabs, src, nblk, sink);
}

// ---- records of 1..1023 B, one lane per record -------------------------------------------------
// A wave takes 64 consecutive records (lane u: record 64b + u, so descriptors and results are
// coalesced) and every lane hashes its own record through the replicated, conflict-free T0..T3:
// no row tree, no shift operators per record.  The record is END-aligned on a FIXED window of NG
// 32-B groups: word i = bytes [e + 4 - 32NG + 4i, +4), built by one v_perm (the lane's byte shift)
// from the aligned dwords of the window.  Bytes before p are zeroed -- the chain starts at 0, so
// leading zeros are free -- and the word holding p injects U[z] (z zeroed bytes), so the state
// entering the record is Value()'s 0xFFFFFFFF.  Loads are 16-B chunks, 4-B aligned, all issued up
// front: a chunk wholly below the record's first aligned dword reads a dummy line shared by every
// such lane (all its bytes are masked), one straddling it reads up to 12 B before it -- so records
// less than 16 B after the base take the slow path, with n == 0 and n > 32 (NG - 1): those lanes are
// hashed after the batch, one record per pass of the whole wave (slow_finish).  A wave pays one
// memory latency per batch of 64 records, and the window is hashed as two chains for ILP (NG = 9:
// groups 0..4 (A) and 5..8 (B, the last 128 B), folded as shift128(A) ^ B, slot 3 = shift 128).
// Groups wholly below every lane's record are skipped (wave-uniform).
// lanerec_window<NG>: the body for a window of NG groups (records of 1..32*(NG-1) B); chain B
// takes the last NG - NA groups, a power of two so the fold is one shift slot.  NG = 9 is the
// <= 256-B class, NG = 17 the 257..512-B class (chain B = 256 B, slot 4).
template <class Src, class Sink, uint32_t NG, uint32_t kWpw = kWavesPerWg, uint32_t kChains = 2,
          bool kPrefetch = false>
__device__ __forceinline__ void lanerec_window(const uint32_t* __restrict__ tabs, Src src, uint64_t nblk,
                                               Sink sink) {
  constexpr uint32_t NA = (NG + 1) / 2, NB = NG - NA, MAXN = 32u * (NG - 1);
  constexpr int kSlotB = NB == 4 ? 3 : (NB == 8 ? 4 : (NB == 16 ? 5 : -1));
  static_assert(kSlotB >= 0, "chain B must span 128, 256 or 512 B");
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  stage_tables<PDB_CAT_TREE16, PDB_CAT_S1024>(lds, tabs);  // slots 0..5 = 16..512 (3 = 128), 6 = 1024
  const uint32_t u = threadIdx.x & 63u;
  const uint32_t ureg = tabs[PDB_UNSHIFT_OFF + (u & 15u)];
  __syncthreads();
  const LaneTabs lt = lane_tabs(u);
  const uintptr_t dummy = reinterpret_cast<uintptr_t>(tabs);  // >= 4 KiB + 256 B of valid bytes
  const uintptr_t lo_ok = reinterpret_cast<uintptr_t>(src.base) + 16u;
  const uint64_t nbat = (nblk + 63u) >> 6;
  const uint64_t W = static_cast<uint64_t>(gridDim.x) * kWpw;
  uint64_t b = static_cast<uint64_t>(blockIdx.x) * kWpw + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (b >= nbat) return;
  auto idx = [&](uint64_t bb) -> uint64_t {
    const uint64_t i = (bb << 6) + u;
    return i < nblk ? i : nblk - 1;
  };
  // the window of one lane's record: chunk h (16 B) at d0 + 16 h; chunks wholly below the record
  // read the dummy line.  Records outside the fast range hash a 1-B stand-in (slow path below).
  auto issue = [&](const BlkDesc& dd, u32x4 (&CC)[2 * NG]) {
    const uintptr_t q0 = reinterpret_cast<uintptr_t>(dd.p);
    const bool f = (dd.n - 1u) <= MAXN - 1u && dd.init_raw == 0xFFFFFFFFu && q0 >= lo_ok;
    const uintptr_t q = f ? q0 : dummy + 16u;
    const uintptr_t a1 = (q + (f ? dd.n : 1u) - 1u) & ~static_cast<uintptr_t>(3);
    const uintptr_t a0 = q & ~static_cast<uintptr_t>(3);
    const uintptr_t w0 = a1 + 4u - 32u * NG;
    CC[0] = u32x4{0, 0, 0, 0};  // dwords 0..3 lie wholly below every record of <= MAXN B
#pragma unroll
    for (uint32_t h = 1; h < 2 * NG; ++h) {
      const uintptr_t a = w0 + 16u * h;
      CC[h] = gload128<false>(a + 12u < a0 ? dummy : a);
    }
  };
  typename Src::Raw raw = src.load(idx(b));
  u32x4 C[2 * NG];
  BlkDesc dnext{};
  if constexpr (kPrefetch) {  // batch b's window now, the loop issues batch b + W's before hashing b
    keep_alive(raw);
    dnext = src.lane(raw);
    issue(dnext, C);
    raw = src.load(idx(b + W < nbat ? b + W : b));
  }
  for (;;) {
    const uint64_t i = (b << 6) + u, bn = b + W;
    BlkDesc d;
    u32x4 Cn[kPrefetch ? 2 * NG : 1];
    if constexpr (kPrefetch) {
      d = dnext;
      keep_alive(raw);
      dnext = src.lane(raw);  // batch bn (clamped past the end: valid, unused)
      issue(dnext, Cn);
      raw = src.load(idx(bn + W < nbat ? bn + W : bn));
    } else {
      keep_alive(raw);
      d = src.lane(raw);
      issue(d, C);
      raw = src.load(idx(bn < nbat ? bn : b));  // next batch's descriptors (unconditional)
    }
    const uintptr_t p0 = reinterpret_cast<uintptr_t>(d.p);
    const bool fast = (d.n - 1u) <= MAXN - 1u && d.init_raw == 0xFFFFFFFFu && p0 >= lo_ok;
    const uint32_t n = fast ? d.n : 1u;
    const uintptr_t e = (fast ? p0 : dummy + 16u) + n;
    const uintptr_t A1 = (e - 1u) & ~static_cast<uintptr_t>(3);
    const bool valid = i < nblk;
    const uint32_t pre = SinkOps<Sink>::pre(sink, idx(b), d);
    const uint32_t sel = static_cast<uint32_t>(e - A1) * 0x01010101u + 0x03020100u;  // bytes sb..sb+3
    const int32_t dz0 = static_cast<int32_t>(32u * NG - n);  // p - start of word W_{-1}
    const uint32_t uz = __shfl(ureg, static_cast<uint32_t>(dz0) & 3u, 64);
    // first group holding a byte of some lane's record (wave-uniform): groups below are all zero
    uint32_t t0 = static_cast<uint32_t>(dz0) >> 5;  // group t holds bytes iff dz0 - 32t < 32
    t0 = fast ? (t0 < NG - 1 ? t0 : NG - 1) : NG - 1;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
      const uint32_t o = __shfl_xor(t0, k, 64);
      t0 = o < t0 ? o : t0;
    }
    t0 = __builtin_amdgcn_readfirstlane(t0);
    auto dw = [&](int k) -> uint32_t {  // dword k of the window (k = -1: before it, always masked)
      if (k < 0) return 0u;
      const u32x4& q = C[k >> 2];
      return (k & 3) == 0 ? q.x : ((k & 3) == 1 ? q.y : ((k & 3) == 2 ? q.z : q.w));
    };
    auto group = [&](uint32_t& c, int t) {
      const int32_t dz = dz0 - 32 * t;
      if (__builtin_amdgcn_ballot_w64(dz >= 0) == 0) {  // the whole group inside every record
#pragma unroll
        for (int k = 0; k < 8; ++k) c = step4(lds, lt, c, __builtin_amdgcn_perm(dw(8 * t + k), dw(8 * t + k - 1), sel));
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int32_t z = dz - 4 * k;
          const uint32_t w = __builtin_amdgcn_perm(dw(8 * t + k), dw(8 * t + k - 1), sel);
          const uint32_t m = z <= 0 ? 0xFFFFFFFFu : (z >= 4 ? 0u : (0xFFFFFFFFu << (8u * static_cast<uint32_t>(z))));
          const uint32_t inj = static_cast<uint32_t>(z) < 4u ? uz : 0u;
          c = step4(lds, lt, c ^ inj, w & m);
        }
      }
    };
    uint32_t c;
    if constexpr (kChains == 2) {
      uint32_t ca = 0, cb = 0;
#pragma unroll
      for (int t = 0; t < static_cast<int>(NA); ++t) {
        if (static_cast<uint32_t>(t) >= t0) group(ca, t);
        if (t + NA < NG && static_cast<uint32_t>(t) + NA >= t0) group(cb, t + NA);
      }
      c = t0 < NA ? shift_op_x(lds, kSlotB, ca, cb) : cb;
    } else {
      // kChains chains: chain 0 = groups [0, L0), chain k >= 1 = the k-th of the last 128-B spans
      // (4 groups each); folded as c = shift128(c) ^ chain_k (linear: a chain wholly below every
      // record is 0 and its fold a no-op, so it is skipped wave-uniformly)
      constexpr int NT = static_cast<int>(kChains) - 1, L0 = static_cast<int>(NG) - 4 * NT;
      static_assert(L0 >= 4, "chain 0 must be the longest");
      uint32_t ch[kChains] = {};
#pragma unroll
      for (int t = 0; t < L0; ++t) {
        if (static_cast<uint32_t>(t) >= t0) group(ch[0], t);
#pragma unroll
        for (int k = 1; k <= NT; ++k)
          if (t < 4 && static_cast<uint32_t>(L0 + 4 * (k - 1) + t) >= t0) group(ch[k], L0 + 4 * (k - 1) + t);
      }
      c = ch[0];
#pragma unroll
      for (int k = 1; k <= NT; ++k)
        c = t0 < static_cast<uint32_t>(L0 + 4 * (k - 1)) ? shift_op_x(lds, 3, c, ch[k]) : ch[k];
    }
    if (valid && fast) SinkOps<Sink>::put(sink, i, c, d, pre);
    // the batch's records outside the fast range, one per pass of the whole wave
    uint64_t slow = __builtin_amdgcn_ballot_w64(valid && !fast);
    const uint32_t plo = static_cast<uint32_t>(p0), phi = static_cast<uint32_t>(static_cast<uint64_t>(p0) >> 32);
    while (slow) {
      const uint32_t k = static_cast<uint32_t>(__builtin_ctzll(slow));
      slow &= slow - 1;
      const uintptr_t sp = static_cast<uintptr_t>(uniform64(__builtin_amdgcn_readlane(plo, k), __builtin_amdgcn_readlane(phi, k)));
      const uint32_t sn = __builtin_amdgcn_readlane(d.n, k);
      SlowFirst sf;
      slow_issue(sf, sp, sn, u, dummy);
      const uint32_t rs = slow_finish(lds, lt, u, ureg, sf, sp, sn);
      const BlkDesc sd{reinterpret_cast<const uint8_t*>(sp), sn, 0xFFFFFFFFu};
      if (u == 0) SinkOps<Sink>::put(sink, (b << 6) + k, rs, sd, __builtin_amdgcn_readlane(pre, k));
    }
    if constexpr (kPrefetch) {
#pragma unroll
      for (uint32_t h = 0; h < 2 * NG; ++h) C[h] = Cn[h];
    }
    if (bn >= nbat) break;
    b = bn;
  }
}

template <class Src, class Sink>
__global__ __launch_bounds__(kThreads) void crc_lanerec9_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                                uint64_t nblk, Sink sink) {
  lanerec_window<Src, Sink, 9>(tabs, src, nblk, sink);
}

// 512 threads (8 waves, one workgroup per CU for the 160-KiB LDS image): 256 VGPRs per lane hold
// the 34 x 16-B window without spilling (1024 threads cap it at 128 and spill ~240 B per lane)
constexpr uint32_t kThreads17 = 512;
template <class Src, class Sink, uint32_t kChains = 4>
__global__ __launch_bounds__(kThreads17) void crc_lanerec17_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                                   uint64_t nblk, Sink sink) {
  lanerec_window<Src, Sink, 17, kThreads17 / 64, kChains>(tabs, src, nblk, sink);
}

uint32_t grid_for(const LaunchGeom& g, uint64_t nblk) {
  const uint64_t want = (nblk + kWavesPerWg - 1) / kWavesPerWg;
  return static_cast<uint32_t>(want < g.grid ? (want ? want : 1) : g.grid);
}



// Records of 513..1024 B (PDB_CRC_SIZE_1023; fixed strides of 513..1023 B): a 33-group (1056-B)
// window, 8 chains, 256 threads (one wave per SIMD: the 66 x 16-B window lives in VGPRs + AGPRs)
template <class Src, class Sink>
__global__ __launch_bounds__(256) void crc_lanerec33_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                            uint64_t nblk, Sink sink) {
  lanerec_window<Src, Sink, 33, 4, 8>(tabs, src, nblk, sink);
}

uint32_t grid_wg(const LaunchGeom& g, uint64_t nblk, uint32_t wg) {
  const uint64_t want = ((nblk + 63) / 64 + wg / 64 - 1) / (wg / 64);
  return static_cast<uint32_t>(want < g.grid ? (want ? want : 1) : g.grid);
}

// crc_lanerec17_kernel: one wave per batch of 64 records, kThreads17 / 64 waves per workgroup
uint32_t grid17(const LaunchGeom& g, uint64_t nblk) {
  const uint64_t want = ((nblk + 63) / 64 + kThreads17 / 64 - 1) / (kThreads17 / 64);
  return static_cast<uint32_t>(want < g.grid ? (want ? want : 1) : g.grid);
}

// One lane per record, the window sized by the class: <= 256 B (9 groups, 1024 threads), 257..512 B
// (17 groups, 512 threads), 513..1023 B (33 groups, 256 threads; the window overflows into AGPRs).
// Records outside the class take the kernel's slow path.
template <class Src, class Sink>
void launch_lanerec(const LaunchGeom& g, const uint32_t* d_tables, const Src& src, uint64_t nblk, uint32_t cls,
                    const Sink& sink, hipStream_t s) {
  if (cls <= 256u)
    hipLaunchKernelGGL((crc_lanerec9_kernel<Src, Sink>), dim3(grid_for(g, (nblk + 63) / 64)), dim3(kThreads), 0, s,
                       d_tables, src, nblk, sink);
  else if (cls <= 512u)
    hipLaunchKernelGGL((crc_lanerec17_kernel<Src, Sink>), dim3(grid17(g, nblk)), dim3(kThreads17), 0, s, d_tables,
                       src, nblk, sink);
  else
    hipLaunchKernelGGL((crc_lanerec33_kernel<Src, Sink>), dim3(grid_wg(g, nblk, 256)), dim3(256), 0, s, d_tables,
                       src, nblk, sink);
}

}  // namespace
}  // namespace pdb
