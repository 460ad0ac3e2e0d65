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

// Fold the 64 lane partials (lane v's partial ends P*(63-v) bytes before the region end, where
// slots 0..5 hold "shift by P << k").  Result valid in lane 0.
__device__ __forceinline__ uint32_t wave_tree(const char* lds, uint32_t lane, uint32_t c) {
#pragma unroll
  for (uint32_t k = 0; k < 6; ++k) {
    const uint32_t y = __shfl_down(c, 1u << k, 64);
    if ((lane & ((2u << k) - 1u)) == 0) c = shift_op(lds, k, c) ^ y;
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
template <int kTree, int kHorner>
__device__ __forceinline__ void stage_tables(char* lds, const uint32_t* __restrict__ tabs) {
  for (uint32_t i = threadIdx.x; i < 4u * 256u * 8u; i += blockDim.x) {
    const uint32_t k = i >> 11, b = (i >> 3) & 255u, part = i & 7u;
    const uint32_t v = tabs[k * 256u + b];
    const uint32_t addr = ((k >> 1) << 16) | (b << 8) | ((k & 1u) << 7) | (part << 4);
    *reinterpret_cast<u32x4*>(lds + addr) = u32x4{v, v, v, v};
  }
  const u32x4* cat = reinterpret_cast<const u32x4*>(tabs + 1024);
  constexpr uint32_t nslots = kHorner >= 0 ? 7u : 6u;
  for (uint32_t i = threadIdx.x; i < nslots * 256u; i += blockDim.x) {
    const uint32_t slot = i >> 8;
    const uint32_t src = slot < 6 ? kTree + slot : static_cast<uint32_t>(kHorner);
    *reinterpret_cast<u32x4*>(lds + PDB_MAIN_BYTES + i * 16u) = cat[src * 256u + (i & 255u)];
  }
}

// 16 dwords of the 64-B chunk at q.  `s` = q & 3 (uniform across the wave for one block).
__device__ __forceinline__ void load_chunk(uint32_t d[16], const uint8_t* q, uint32_t s) {
  if (s == 0) {
    const u32x4a4* v = reinterpret_cast<const u32x4a4*>(q);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u32x4a4 x = v[i];
      d[4 * i + 0] = x.x;
      d[4 * i + 1] = x.y;
      d[4 * i + 2] = x.z;
      d[4 * i + 3] = x.w;
    }
  } else {
    const uint8_t* a = q - s;
    const u32x4a4* v = reinterpret_cast<const u32x4a4*>(a);
    uint32_t e[17];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u32x4a4 x = v[i];
      e[4 * i + 0] = x.x;
      e[4 * i + 1] = x.y;
      e[4 * i + 2] = x.z;
      e[4 * i + 3] = x.w;
    }
    e[16] = *reinterpret_cast<const uint32_t*>(a + 64);
#pragma unroll
    for (int i = 0; i < 16; ++i) d[i] = __builtin_amdgcn_alignbyte(e[i + 1], e[i], s);
  }
}

__device__ __forceinline__ uint32_t chain16(const char* lds, const LaneTabs& lt, uint32_t c,
                                            const uint32_t d[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) c = step4(lds, lt, c, d[i]);
  return c;
}

// Raw state S(init_raw, p[0..n)) in lane 0 for one block of any length/alignment.
__device__ uint32_t crc_block(const char* lds, const LaneTabs& lt, uint32_t lane, const uint8_t* p,
                              uint32_t n, uint32_t init_raw) {
  const uint32_t t = n & 63u;
  const uint32_t K = n >> 6;
  uint32_t c = 0;
  if (lane == 0) {
    c = init_raw;
    uint32_t i = 0;
    for (; i < (t & 3u); ++i) c = step1(lds, lt, c, p[i]);
    for (; i < t; i += 4) c = step4(lds, lt, c, ld32u(p + i));
  }
  if (K == 0) return c;
  const uint8_t* q0 = p + t;
  const uint32_t s = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(q0) & 3u);
  const uint32_t R = (K + 63u) >> 6;
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t ch = lane + (r << 6);
    if (ch < K) {
      if (r) c = shift_op(lds, PDB_SLOT_HORNER, c);
      uint32_t d[16];
      load_chunk(d, q0 + static_cast<uint64_t>(ch) * 64u, s);
      c = chain16(lds, lt, c, d);
    }
  }
  const uint32_t q = K & 63u;
  if (q) c = __shfl(c, (lane + q) & 63u, 64);
  return wave_tree(lds, lane, c);
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

template <int kNP>
__device__ __forceinline__ uint32_t hash4k(const char* lds, const LaneTabs& lt, uint32_t lane,
                                           uint32_t c, const u32x4 (&v)[4]) {
  const uint32_t d[16] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                          v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
  constexpr int per = 16 / kNP;  // dwords per piece
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i && (i % per) == 0) c = shift_op(lds, PDB_SLOT_HORNER, c);
    c = step4(lds, lt, c, d[i]);
  }
  return wave_tree(lds, lane, c);
}

template <int kNP, int kDepth>
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
  constexpr int kHorner = kNP == 1 ? -1 : (kNP == 2 ? PDB_CAT_H2016 : PDB_CAT_H1008);
  stage_tables<kTree, kHorner>(lds, tabs);
  __syncthreads();
  const LaneTabs lt = lane_tabs(lane);
  const uint32_t init_raw = (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu;
  for (uint64_t b = b0; b < nblk; b += kDepth * nw) {
#pragma unroll
    for (int k = 0; k < kDepth; ++k) {
      const uint64_t bk = b + k * nw;
      if (bk >= nblk) return;  // wave-uniform
      u32x4 cur[4] = {buf[k][0], buf[k][1], buf[k][2], buf[k][3]};
      const uint64_t bn = bk + kDepth * nw;
      load4k<kNP>(buf[k], base, stride, bn < nblk ? bn : bk, lane);  // clamp: valid block
      const uint32_t c = hash4k<kNP>(lds, lt, lane, lane == 0 ? init_raw : 0u, cur);
      if (lane == 0) out[bk] = finalize(c, flags);
    }
  }
}

// ---- fixed-stride batch, generic (any length / alignment) ---------------------------------------
__global__ __launch_bounds__(kThreads) void crc_fixed_kernel(
    const uint32_t* __restrict__ tabs, const uint8_t* __restrict__ base, uint64_t stride,
    uint32_t len, uint64_t nblk, uint32_t flags, uint32_t init, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  stage_tables<PDB_CAT_TREE64, PDB_CAT_H4032>(lds, tabs);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const LaneTabs lt = lane_tabs(lane);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * kWavesPerWg;
  const uint32_t init_raw = (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu;
  for (uint64_t b = wave_id_uniform(); b < nblk; b += nwaves) {
    const uint32_t c = crc_block(lds, lt, lane, base + b * stride, len, init_raw);
    if (lane == 0) out[b] = finalize(c, flags);
  }
}

// ---- descriptor batch (variable length, any alignment); optional verify ---------------------
template <int kMode>
__global__ __launch_bounds__(kThreads) void crc_desc_kernel(
    const uint32_t* __restrict__ tabs, const uint8_t* __restrict__ base,
    const pdb_blk* __restrict__ blk, uint64_t nblk, uint32_t flags,
    const uint32_t* __restrict__ expected, uint32_t* __restrict__ out, uint8_t* __restrict__ ok,
    uint32_t* __restrict__ nbad) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  stage_tables<PDB_CAT_TREE64, PDB_CAT_H4032>(lds, tabs);
  __syncthreads();

  const uint32_t lane = threadIdx.x & 63u;
  const LaneTabs lt = lane_tabs(lane);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * kWavesPerWg;
  for (uint64_t i = wave_id_uniform(); i < nblk; i += nwaves) {
    const pdb_blk d = blk[i];
    const uint32_t init_raw = (flags & PDB_CRC_USE_INIT) ? ~d.init : 0xFFFFFFFFu;
    const uint32_t c = crc_block(lds, lt, lane, base + d.off, d.len, init_raw);
    if (lane == 0) {
      const uint32_t v = finalize(c, flags);
      if constexpr (kMode == kModeOut) {
        out[i] = v;
      } else {
        const bool good = (v == expected[i]);
        if (ok) ok[i] = good ? 1 : 0;
        if (!good && nbad) atomicAdd(nbad, 1u);
      }
    }
  }
}

// ---- sstable trailers: seal (write) or verify (read) ----------------------------------------
template <bool kSeal>
__global__ __launch_bounds__(kThreads) void sst_kernel(const uint32_t* __restrict__ tabs,
                                                        uint8_t* __restrict__ buf,
                                                        const pdb_block_handle* __restrict__ h,
                                                        uint64_t n, uint8_t* __restrict__ ok,
                                                        uint32_t* __restrict__ nbad) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  stage_tables<PDB_CAT_TREE64, PDB_CAT_H4032>(lds, tabs);
  __syncthreads();

  const uint32_t lane = threadIdx.x & 63u;
  const LaneTabs lt = lane_tabs(lane);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * kWavesPerWg;
  for (uint64_t i = wave_id_uniform(); i < n; i += nwaves) {
    const pdb_block_handle hd = h[i];
    uint8_t* p = buf + hd.offset;
    // CRC input = contents || type byte  (table/table_builder.cc:197-198; format.cc:98)
    const uint32_t c = crc_block(lds, lt, lane, p, static_cast<uint32_t>(hd.size + 1), 0xFFFFFFFFu);
    if (lane == 0) {
      uint8_t* tr = p + hd.size + 1;
      if constexpr (kSeal) {
        const uint32_t m = pdb_mask(~c);  // EncodeFixed32(trailer+1, Mask(crc))
        tr[0] = static_cast<uint8_t>(m);
        tr[1] = static_cast<uint8_t>(m >> 8);
        tr[2] = static_cast<uint8_t>(m >> 16);
        tr[3] = static_cast<uint8_t>(m >> 24);
      } else {
        const uint32_t stored = static_cast<uint32_t>(tr[0]) | (static_cast<uint32_t>(tr[1]) << 8) |
                                (static_cast<uint32_t>(tr[2]) << 16) |
                                (static_cast<uint32_t>(tr[3]) << 24);
        const bool good = pdb_unmask(stored) == ~c;
        if (ok) ok[i] = good ? 1 : 0;
        if (!good && nbad) atomicAdd(nbad, 1u);
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
template <int kPat, int kDepth, int kAssign>
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
  for (uint64_t b = first; b < last; b += step * kDepth) {
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
    hipLaunchKernelGGL(crc_fixed_kernel, grid, block, 0, s, d_tables, base, stride, len, nblk,
                       flags, init, out);
    return hipGetLastError();
  }
#define PDB_FAST(NP, D)                                                                      \
  hipLaunchKernelGGL((crc_fast4k_kernel<NP, D>), grid, block, 0, s, d_tables, base, stride, nblk, \
                     flags, init, out)
  switch (g_fast_variant) {
    case 1: PDB_FAST(1, 1); break;
    case 2: PDB_FAST(4, 1); break;
    default: PDB_FAST(2, 1); break;  // measured best: 2 x 32-B pieces per lane, depth 1
  }
#undef PDB_FAST
  return hipGetLastError();
}

hipError_t launch_desc(const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                       const pdb_blk* blk, uint64_t nblk, uint32_t flags, int mode,
                       const uint32_t* expected, uint32_t* out, uint8_t* ok, uint32_t* nbad,
                       hipStream_t s) {
  if (nblk == 0) return hipSuccess;
  const dim3 grid(grid_for(g, nblk)), block(kThreads);
  if (mode == kModeOut)
    hipLaunchKernelGGL(crc_desc_kernel<kModeOut>, grid, block, 0, s, d_tables, base, blk, nblk,
                       flags, expected, out, ok, nbad);
  else
    hipLaunchKernelGGL(crc_desc_kernel<kModeVerify>, grid, block, 0, s, d_tables, base, blk, nblk,
                       flags, expected, out, ok, nbad);
  return hipGetLastError();
}

hipError_t launch_sst(const LaunchGeom& g, const uint32_t* d_tables, uint8_t* buf, uint64_t buf_len,
                      const pdb_block_handle* h, uint64_t n, bool seal, uint8_t* ok, uint32_t* nbad,
                      hipStream_t s) {
  (void)buf_len;
  if (n == 0) return hipSuccess;
  const dim3 grid(grid_for(g, n)), block(kThreads);
  if (seal)
    hipLaunchKernelGGL(sst_kernel<true>, grid, block, 0, s, d_tables, buf, h, n, ok, nbad);
  else
    hipLaunchKernelGGL(sst_kernel<false>, grid, block, 0, s, d_tables, buf, h, n, ok, nbad);
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
