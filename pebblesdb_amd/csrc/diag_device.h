// diag_device.h -- A/B kernel variants of the diagnostics library (libpdb_crc32c_diag.so) only.
// These are the alternatives measured against the shipped kernels (profiles/r01_ab_*);
// the product library (libpdb_crc32c.so) never instantiates them.
#pragma once
#include "crc32c_device.h"

namespace pdb {
namespace {

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

// ---- quad-transposed 4-KiB geometry -------------------------------------------------------------
// The coalesced loads leave lane u = 4m + b with the 16-B pieces at 16u + 1024j (j = 0..3): four
// chains that must be folded with three "shift 1024/2048" operator lookups per lane (single-copy
// LDS tables, ~3 cycles of bank conflicts per lookup).  A 4x4 transpose of 16-B elements inside
// each quad (two DPP butterfly stages, quad_perm xor 1 / xor 2) gives lane (m, b) instead the 64
// CONTIGUOUS bytes at 1024b + 64m, hashed as one 16-step chain through the replicated,
// conflict-free T0..T3 -- no per-lane fold at all; the tree's levels become "shift 1024" (bit 0 of
// the lane = b), "shift 2048" (bit 1), then 64, 128, 256, 512 (m): same op count as before.
// One butterfly stage on the register pair (A, B) = (R[j], R[j ^ K]): the lane with bit K clear
// keeps A and takes its partner's A into B; the lane with bit K set keeps B and takes its
// partner's B into A.
template <int kCtrl>
__device__ __forceinline__ void quad_swap(u32x4& A, u32x4& B, bool hi) {
  const u32x4 snd = hi ? A : B;
  u32x4 rcv;
  rcv.x = __builtin_amdgcn_mov_dpp(snd.x, kCtrl, 0xF, 0xF, true);
  rcv.y = __builtin_amdgcn_mov_dpp(snd.y, kCtrl, 0xF, 0xF, true);
  rcv.z = __builtin_amdgcn_mov_dpp(snd.z, kCtrl, 0xF, 0xF, true);
  rcv.w = __builtin_amdgcn_mov_dpp(snd.w, kCtrl, 0xF, 0xF, true);
  A = hi ? rcv : A;
  B = hi ? B : rcv;
}

__device__ __forceinline__ void quad_transpose(u32x4 (&R)[4], uint32_t lane) {
  const bool h1 = (lane & 1u) != 0, h2 = (lane & 2u) != 0;
  quad_swap<0xB1>(R[0], R[1], h1);  // quad_perm [1,0,3,2]: partner lane ^ 1
  quad_swap<0xB1>(R[2], R[3], h1);
  quad_swap<0x4E>(R[0], R[2], h2);  // quad_perm [2,3,0,1]: partner lane ^ 2
  quad_swap<0x4E>(R[1], R[3], h2);
}

// One 16-step chain over 64 contiguous bytes (4 x u32x4 in order) from `start`.
__device__ __forceinline__ uint32_t chain64(const char* lds, const LaneTabs& lt, uint32_t start, const u32x4 (&R)[4]) {
  const uint32_t w[16] = {R[0].x, R[0].y, R[0].z, R[0].w, R[1].x, R[1].y, R[1].z, R[1].w,
                          R[2].x, R[2].y, R[2].z, R[2].w, R[3].x, R[3].y, R[3].z, R[3].w};
  uint32_t x = start ^ w[0];
#pragma unroll
  for (int i = 1; i <= 16; ++i) x = step4x(lds, lt, x, i < 16 ? w[i] : 0u);
  return x;
}

// The same 64 bytes as two independent 8-step chains folded with "shift 32" (slot 6): ILP 2 for
// one operator lookup per lane.
__device__ __forceinline__ uint32_t chain64x2(const char* lds, const LaneTabs& lt, uint32_t start,
                                              const u32x4 (&R)[4]) {
  const uint32_t a[8] = {R[0].x, R[0].y, R[0].z, R[0].w, R[1].x, R[1].y, R[1].z, R[1].w};
  const uint32_t b[8] = {R[2].x, R[2].y, R[2].z, R[2].w, R[3].x, R[3].y, R[3].z, R[3].w};
  uint32_t xa = start ^ a[0], xb = b[0];
#pragma unroll
  for (int i = 1; i <= 8; ++i) {
    xa = step4x(lds, lt, xa, i < 8 ? a[i] : 0u);
    xb = step4x(lds, lt, xb, i < 8 ? b[i] : 0u);
  }
  return shift_op_x(lds, PDB_SLOT_HORNER, xa, xb);
}

// kPair: the wave hashes blocks two at a time (8 independent chains, next pair's 8 KiB in flight)
// -- the ILP that lets 8 waves per CU (kWaves = 8, the nt loads' best shape) hide LDS latency.
// kXcd: workgroups are dispatched to the 8 XCDs round-robin (blockIdx.x % 8); kXcd renumbers
// them so each XCD's CUs own consecutive 64-KiB block windows (A/B diagnostics).
template <int kSync, int kNP = 2, bool kNT = false, int kWaves = kWavesPerWg, bool kPair = false,
          bool kXcd = false, int kQuad = 0, bool kPrio = false>
__global__ __launch_bounds__(kWaves * 64) void crc_pack4k_ab_kernel(
    const uint32_t* __restrict__ tabs, const uint8_t* __restrict__ base, uint64_t stride,
    uint64_t nblk, uint32_t flags, uint32_t init, uint32_t* __restrict__ out) {
  static_assert(kNP == 2 || kNP == 4, "lane pieces: 2 x 32 B or 4 x 16 B");
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  const uint32_t u = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  const uint32_t wg = (kXcd && (gridDim.x & 7u) == 0) ? (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)
                                                       : blockIdx.x;
  const uint64_t w = static_cast<uint64_t>(wg) * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u32x4 buf[4], buf2[4];
  load4k<kNP, kNT>(buf, base, stride, w < nblk ? w : nblk - 1, u);
  if constexpr (kPair) load4k<kNP, kNT>(buf2, base, stride, w + nw < nblk ? w + nw : nblk - 1, u);
  if constexpr (kNP == 4)
    stage_tables<PDB_CAT_TREE16, kQuad == 2 ? 1 : PDB_CAT_S1024, PDB_CAT_S2048, false, kQuad != 0>(lds, tabs);
  else
    stage_tables<PDB_CAT_TREE32, PDB_CAT_S2048>(lds, tabs);
  __syncthreads();
  if (kSync == 0 && w >= nblk) return;
  const LaneTabs lt = lane_tabs(u);
  const uint32_t init_raw = (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu;
  const uint32_t c0 = u == 0 ? init_raw : 0u;
  uint32_t res = 0, it = 0;
  // kSync: the workgroup's 16 waves (16 consecutive blocks) stay in lock step, one barrier per
  // 4-block group, so their outstanding loads cover one compact 64-KiB span at a time.
  const uint64_t wg_first = static_cast<uint64_t>(wg) * kWaves;
  if (kSync > 0 && wg_first >= nblk) return;
  uint32_t grp = 0;
  uint64_t win0 = w;
  for (uint64_t g = w, gw = wg_first; (kSync > 0 ? gw : g) < nblk; g += 4 * nw, gw += 4 * nw) {
    if constexpr (kSync > 0) {
      if ((grp++ % kSync) == 0) __syncthreads();
    }
    uint32_t p[4];
    if constexpr (kPair) {
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const uint64_t bk = g + r * nw;
        u32x4 cur[4] = {buf[0], buf[1], buf[2], buf[3]};
        u32x4 cur2[4] = {buf2[0], buf2[1], buf2[2], buf2[3]};
        const uint64_t bn = bk + 2 * nw;
        if (bn < nblk) load4k<kNP, kNT>(buf, base, stride, bn, u);  // wave-uniform
        if (bn + nw < nblk) load4k<kNP, kNT>(buf2, base, stride, bn + nw, u);
        p[r] = bk < nblk ? partial4k<kNP>(lds, lt, c0, cur) : 0u;
        p[r + 1] = bk + nw < nblk ? partial4k<kNP>(lds, lt, c0, cur2) : 0u;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint64_t bk = g + r * nw;
        u32x4 cur[4] = {buf[0], buf[1], buf[2], buf[3]};
        const uint64_t bn = bk + nw;
        if constexpr (kPrio) __builtin_amdgcn_s_setprio(2);  // A/B: issue the next block's loads first
        if (bn < nblk) load4k<kNP, kNT>(buf, base, stride, bn, u);  // wave-uniform
        if constexpr (kPrio) __builtin_amdgcn_s_setprio(0);
        if constexpr (kQuad != 0) {
          static_assert(kNP == 4, "the quad transpose needs 4 x 16-B lane pieces");
          quad_transpose(cur, u);
          if constexpr (kQuad == 1)
            p[r] = bk < nblk ? chain64(lds, lt, c0, cur) : 0u;
          else
            p[r] = bk < nblk ? chain64x2(lds, lt, c0, cur) : 0u;
        } else {
          p[r] = bk < nblk ? partial4k<kNP>(lds, lt, c0, cur) : 0u;
        }
      }
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

template <class Src, class Sink, bool kNT>
__global__ __launch_bounds__(kThreads) void crc_sst4k_nofold_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                                    uint64_t nblk, Sink sink) {
  sized_kernel_body<Src, Sink, kNT, 4, true>(tabs, src, nblk, sink);
}

template <class Src, class Sink, bool kNT>
__global__ __launch_bounds__(kThreads) void crc_rec256_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                              uint64_t nblk, Sink sink) {
  sized_kernel_body<Src, Sink, kNT, 0, false, 4>(tabs, src, nblk, sink);
}

// ---- records of 1..256 B, one lane per record -------------------------------------------------
// A wave takes 64 consecutive records (lane u: record 64b + u, so descriptors and results are
// coalesced) and every lane hashes its own record as ONE slice-by-4 chain through the replicated,
// conflict-free T0..T3: no row tree, no shift operators (a 132-B WAL record is 33 chain steps of
// one lane, not 16 lanes' pieces plus a 4-level tree of single-copy operator lookups).
// The record is END-aligned on a grid of G 32-B groups (G = ceil((n + 4) / 32), the wave's max):
// word i = bytes [e + 4 - 32G + 4i, +4), i = 0 .. 8G - 2, built by one v_perm (the lane's byte
// shift) from the dwords D[k] at A1 + 4 - 32G + 4k, A1 = the record's last aligned dword.  Bytes
// before p are zeroed -- the chain starts at 0, so leading zeros are free -- and the word holding p
// injects U[z] (z zeroed bytes), so the state entering the record is Value()'s 0xFFFFFFFF.
// Loads are 16-B chunks, 4-B aligned: a chunk wholly below the record's first aligned dword reads
// a dummy (all its bytes are masked), one straddling it reads up to 12 B before it -- so records
// less than 16 B after the base take the slow path, with n == 0 and n > 256: those lanes are
// hashed after the batch, one record per pass of the whole wave (slow_finish).  Value() seeds only
// (the launchers route Extend seeds elsewhere).
template <class Src, class Sink, bool kNT>
__global__ __launch_bounds__(kThreads) void crc_lanerec_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                               uint64_t nblk, Sink sink) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  stage_tables<PDB_CAT_TREE16, PDB_CAT_S1024>(lds, tabs);  // slow path: slots 0..5 = 16..512, 6 = 1024
  const uint32_t u = threadIdx.x & 63u;
  const uint32_t ureg = tabs[PDB_UNSHIFT_OFF + (u & 15u)];
  __syncthreads();
  const LaneTabs lt = lane_tabs(u);
  const uintptr_t dummy = reinterpret_cast<uintptr_t>(tabs);  // >= 4 KiB + 256 B of valid bytes
  const uintptr_t lo_ok = reinterpret_cast<uintptr_t>(src.base) + 16u;
  const uint64_t nbat = (nblk + 63u) >> 6;
  const uint64_t W = static_cast<uint64_t>(gridDim.x) * kWavesPerWg;
  uint64_t b = wave_id_uniform();
  if (b >= nbat) return;
  auto idx = [&](uint64_t bb) -> uint64_t {
    const uint64_t i = (bb << 6) + u;
    return i < nblk ? i : nblk - 1;
  };
  typename Src::Raw raw = src.load(idx(b));
  for (;;) {
    const uint64_t i = (b << 6) + u, bn = b + W;
    keep_alive(raw);
    const BlkDesc d = src.lane(raw);
    raw = src.load(idx(bn < nbat ? bn : b));  // next batch's descriptors (unconditional)
    const bool valid = i < nblk;
    const uint32_t pre = SinkOps<Sink>::pre(sink, idx(b), d);
    const uintptr_t p0 = reinterpret_cast<uintptr_t>(d.p);
    const bool fast = (d.n - 1u) <= 255u && d.init_raw == 0xFFFFFFFFu && p0 >= lo_ok;
    const uintptr_t p = fast ? p0 : dummy + 16u;
    const uint32_t n = fast ? d.n : 1u;
    const uintptr_t e = p + n;
    const uintptr_t A1 = (e - 1u) & ~static_cast<uintptr_t>(3);
    const uintptr_t A0 = p & ~static_cast<uintptr_t>(3);
    const uint32_t sel = static_cast<uint32_t>(e - A1) * 0x01010101u + 0x03020100u;  // bytes sb..sb+3
    uint32_t G = (n + 35u) >> 5;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
      const uint32_t o = __shfl_xor(G, k, 64);
      G = o > G ? o : G;
    }
    G = __builtin_amdgcn_readfirstlane(G);
    const uintptr_t d0 = A1 + 4u - 32u * static_cast<uintptr_t>(G);
    // dz = p - (start of the word): word W_{8t-1} (first of iteration t) has 32G - n - 32t
    int32_t dz = static_cast<int32_t>(32u * G - n);
    const uint32_t uz = __shfl(ureg, static_cast<uint32_t>(dz) & 3u, 64);
    auto issue = [&](u32x4 (&g)[2], uint32_t t) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uintptr_t a = d0 + 32u * t + 16u * h;
        g[h] = gload128<kNT>(a + 12u < A0 ? dummy : a);
      }
    };
    u32x4 nx[2];
    issue(nx, 0);
    uint32_t c = 0, carry = 0;
    for (uint32_t t = 0; t < G; ++t) {
      const u32x4 g0 = nx[0], g1 = nx[1];
      issue(nx, t + 1 < G ? t + 1 : t);  // the last group re-reads itself (unconditional)
      const uint32_t D[9] = {carry, g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      carry = g1.w;
      if (__builtin_amdgcn_ballot_w64(dz >= 0) == 0) {  // the whole group inside every record
#pragma unroll
        for (int k = 0; k < 8; ++k) c = step4(lds, lt, c, __builtin_amdgcn_perm(D[k + 1], D[k], sel));
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int32_t z = dz - 4 * k;
          const uint32_t w = __builtin_amdgcn_perm(D[k + 1], D[k], sel);
          const uint32_t m = z <= 0 ? 0xFFFFFFFFu : (z >= 4 ? 0u : (0xFFFFFFFFu << (8u * static_cast<uint32_t>(z))));
          const uint32_t inj = static_cast<uint32_t>(z) < 4u ? uz : 0u;
          c = step4(lds, lt, c ^ inj, w & m);
        }
      }
      dz -= 32;
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
    if (bn >= nbat) break;
    b = bn;
  }
}

// Four lanes per record (A/B variants 57/58): the lane-per-record kernels are TA-bound (one cache
// line per lane per load), so here a record's window of 16 R 16-B chunks is loaded with
// its chunks interleaved across 4 lanes (lane j: chunks 4m + j), i.e. 64 contiguous bytes of one
// record per lane quad per instruction.  Lane j hashes each of its chunks from 0 and folds
// c = shift64(c) ^ t; the quad is folded with shift16 / shift32.  The dword before a chunk (for the
// byte-shift v_perm) comes from the previous lane of the quad (one bpermute per round).
template <class Src, class Sink, uint32_t R, uint32_t MAXN>
__global__ __launch_bounds__(kThreads) void crc_quadrec_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                              uint64_t nblk, Sink sink) {
  static_assert(MAXN + 4u <= 64u * R, "window too short");
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  stage_tables<PDB_CAT_TREE16, PDB_CAT_S1024>(lds, tabs);  // slots 0..5 = 16..512, 6 = 1024
  const uint32_t u = threadIdx.x & 63u, j = u & 3u;
  const uint32_t ureg = tabs[PDB_UNSHIFT_OFF + (u & 15u)];
  __syncthreads();
  const LaneTabs lt = lane_tabs(u);
  const uintptr_t dummy = reinterpret_cast<uintptr_t>(tabs);
  const uintptr_t lo_ok = reinterpret_cast<uintptr_t>(src.base) + 16u;
  const uint64_t nbat = (nblk + 15u) >> 4;
  const uint64_t W = static_cast<uint64_t>(gridDim.x) * kWavesPerWg;
  uint64_t b = wave_id_uniform();
  if (b >= nbat) return;
  auto idx = [&](uint64_t bb) -> uint64_t {
    const uint64_t i = (bb << 4) + (u >> 2);
    return i < nblk ? i : nblk - 1;
  };
  const uint32_t from = (u & ~3u) | ((j + 3u) & 3u);  // previous lane of the quad (lane 3 for lane 0)
  typename Src::Raw raw = src.load(idx(b));
  for (;;) {
    const uint64_t i = (b << 4) + (u >> 2), bn = b + W;
    keep_alive(raw);
    const BlkDesc d = src.lane(raw);
    const uintptr_t p0 = reinterpret_cast<uintptr_t>(d.p);
    const bool fast = (d.n - 1u) <= MAXN - 1u && d.init_raw == 0xFFFFFFFFu && p0 >= lo_ok;
    const uintptr_t p = fast ? p0 : dummy + 16u;
    const uint32_t n = fast ? d.n : 1u;
    const uintptr_t e = p + n;
    const uintptr_t A1 = (e - 1u) & ~static_cast<uintptr_t>(3);
    const uintptr_t A0 = p & ~static_cast<uintptr_t>(3);
    const uintptr_t ws = A1 + 4u - 64u * R;
    u32x4 C[R];
#pragma unroll
    for (uint32_t m = 0; m < R; ++m) {
      const uintptr_t a = ws + 64u * m + 16u * j;
      C[m] = gload128<false>(a + 12u < A0 ? dummy : a);
    }
    raw = src.load(idx(bn < nbat ? bn : b));
    const bool valid = i < nblk;
    const uint32_t pre = SinkOps<Sink>::pre(sink, idx(b), d);
    const uint32_t sel = static_cast<uint32_t>(e - A1) * 0x01010101u + 0x03020100u;
    const int32_t dz0 = static_cast<int32_t>(64u * R - n);  // p - start of constructed word 0
    const uint32_t uz = __shfl(ureg, static_cast<uint32_t>(dz0) & 3u, 64);
    uint32_t c = 0;
#pragma unroll
    for (uint32_t m = 0; m < R; ++m) {
      const uint32_t send = j < 3u ? C[m].w : (m ? C[m - 1].w : 0u);
      const uint32_t prev = __shfl(send, from, 64);
      const int32_t zc = dz0 - static_cast<int32_t>(16u * (4u * m + j));  // z of the chunk's first word
      if (__builtin_amdgcn_ballot_w64(zc < 16) == 0) continue;  // the round lies below every record
      const uint32_t dw[5] = {prev, C[m].x, C[m].y, C[m].z, C[m].w};
      uint32_t t = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int32_t z = zc - 4 * k;
        const uint32_t w = __builtin_amdgcn_perm(dw[k + 1], dw[k], sel);
        const uint32_t mk = z <= 0 ? 0xFFFFFFFFu : (z >= 4 ? 0u : (0xFFFFFFFFu << (8u * static_cast<uint32_t>(z))));
        const uint32_t inj = static_cast<uint32_t>(z) < 4u ? uz : 0u;
        t = step4(lds, lt, t ^ inj, w & mk);
      }
      c = shift_op_x(lds, 2, c, t);  // c = shift64(c) ^ t
    }
    uint32_t y = __shfl_down(c, 1, 64);
    if ((j & 1u) == 0) c = shift_op_x(lds, 0, c, y);
    y = __shfl_down(c, 2, 64);
    if (j == 0) c = shift_op_x(lds, 1, c, y);
    if (valid && fast && j == 0) SinkOps<Sink>::put(sink, i, c, d, pre);
    uint64_t slow = __builtin_amdgcn_ballot_w64(valid && !fast && j == 0);
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
      if (u == 0) SinkOps<Sink>::put(sink, (b << 4) + (k >> 2), rs, sd, __builtin_amdgcn_readlane(pre, k));
    }
    if (bn >= nbat) break;
    b = bn;
  }
}

// A/B variants: the window of batch b + W issued before batch b is hashed (two windows live):
// 9 groups at 512 threads (variant 55), 17 groups at 256 threads (variant 56, AGPRs available)
template <class Src, class Sink, uint32_t NG, uint32_t kWg>
__global__ __launch_bounds__(kWg) void crc_lanerec_pf_kernel(const uint32_t* __restrict__ tabs, Src src,
                                                             uint64_t nblk, Sink sink) {
  lanerec_window<Src, Sink, NG, kWg / 64, NG == 17 ? 4 : 2, true>(tabs, src, nblk, sink);
}

}  // namespace
}  // namespace pdb
