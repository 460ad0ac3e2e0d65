// crc32c_kernels.hip -- CRC32C (Castagnoli) over batches of independent sstable blocks on
// MI355X (gfx950, CDNA4).  Hand-written HIP; no MFMA (GF(2) byte work is not a contraction).
//
// Replaces the per-block software CRC of the reference: crc32c::Extend -> crc32_software ->
// crc32c_sb8_64_bit (util/crc32c.cc:25-32, 101-103, 585-625), called once per block by
// TableBuilder::WriteRawBlock (table/table_builder.cc:197-199) and ReadBlock
// (table/format.cc:96-98).  Results are bit-identical (tests/golden + oracle parity).
//
// Shipped launches (the kernels themselves live in crc32c_device.h):
//   * crc_pack4k_kernel -- fixed stride, 4-KiB, 16-B aligned blocks (BASELINE configs
//     2/4).  One wave per block, lane l owns four 16-B pieces (16l + 1024j, so every load
//     instruction reads 1 KiB contiguous, non-temporal) hashed as four independent slice-by-4
//     chains, 4 blocks per wave-iteration folded in one packed tree, one barrier per 4-block
//     group keeps the workgroup's 16 waves on 16 consecutive blocks.
//   * crc_stream_kernel / crc_stream16_kernel -- any length / alignment (fixed stride, descriptor
//     lists, sstable seal / verify): 4-KiB rounds of 32-B (or 16-B, nt) lane pieces with per-lane
//     Horner shifts, a broadcast head, lane rotation, packed 4-block trees, one-item-ahead
//     prefetch, and workgroup-local dynamic block scheduling from an LDS counter.
//   * crc_sst4k_kernel -- sstable-sized blocks (4096..4352 B: every data block TableBuilder
//     emits, contents + type): the block's last 4 KiB hashed with the 4-KiB path's geometry, the
//     leading 0..256 B of 4 blocks hashed together as zero-padded pieces from an "unshifted"
//     seed; other lengths in the same launch take a whole-wave slow path.
//   * crc_server_kernel (crc32c_server.hip) -- the persistent scalar Extend service.
// LDS image (crc32c_device.h, "lane-quarter table image"): T0..T3 and the per-lane Horner
// operators (shift 1024, and 2048 or 1008) in 8 replicas each, every lookup bank-conflict free,
// plus the tree operators in single-copy slots; one 1024-thread workgroup per CU stages it once
// and walks blocks persistently.  (Round 1 replicated T0..T3 32x in 128 KiB and left the Horner
// operators in single copies: 3 extra LDS cycles per operator lookup.)  DESIGN.md §3-§6 has the
// measurements.
#include "crc32c_device.h"
#include "crc32c_lanespan.h"

namespace pdb {
namespace {

// ---- long spans: parallel segments + one-workgroup tree combine ------------------------------
// A span of n bytes = a head leaf (n mod S bytes, hashed from the Extend seed) followed by nf
// full segments of S = 2^seg_log2 bytes (hashed from state 0 by the batch kernels, one wave
// each).  The nf + 1 raw leaf states are left-padded with zero leaves to M = 2^m (zero leaves are
// free: R(0^k || X) = R(X) from state 0) and folded by a log2(M)-level tree whose level-k
// operator is "shift S * 2^k" (staged in LDS from the power-of-two catalog); the root is the raw
// state of the whole span, so Extend = ~root.  Leaf i's raw state arrives complemented (the
// batch kernels emit ~state), hence the ~ when loading.
struct SpanGeom {
  uint32_t seg_log2, m_log2;
  uint64_t nf, head;
};

__host__ __device__ inline SpanGeom span_geom(uint64_t n, uint32_t min_seg_log2 = PDB_SPAN_MIN_SEG_LOG2) {
  SpanGeom g;
  g.seg_log2 = min_seg_log2;
  while ((n >> g.seg_log2) + 1 > (1ull << PDB_SPAN_MAX_SEGS_LOG2)) ++g.seg_log2;
  g.nf = n >> g.seg_log2;
  g.head = n & ((1ull << g.seg_log2) - 1);
  g.m_log2 = 0;
  while ((1ull << g.m_log2) < g.nf + 1) ++g.m_log2;
  return g;
}

__global__ __launch_bounds__(1024) void span_combine_kernel(const uint32_t* __restrict__ pow2,
                                                            const uint32_t* __restrict__ leaves,
                                                            uint32_t seg_log2, uint32_t m_log2,
                                                            uint64_t nleaves, uint32_t* __restrict__ out) {
  __shared__ uint32_t sw[1u << PDB_SPAN_MAX_SEGS_LOG2];
  __shared__ uint32_t ops[PDB_SPAN_MAX_SEGS_LOG2][1024];
  const uint32_t M = 1u << m_log2;
  for (uint32_t i = threadIdx.x; i < m_log2 * 1024u; i += blockDim.x)
    ops[i >> 10][i & 1023u] = pow2[(seg_log2 + (i >> 10)) * 1024u + (i & 1023u)];
  const uint32_t pad = M - static_cast<uint32_t>(nleaves);
  for (uint32_t i = threadIdx.x; i < M; i += blockDim.x) sw[i] = i < pad ? 0u : ~leaves[i - pad];
  __syncthreads();
  for (uint32_t k = 0; k < m_log2; ++k) {
    const uint32_t half = 1u << k, pairs = M >> (k + 1);
    for (uint32_t j = threadIdx.x; j < pairs; j += blockDim.x) {
      const uint32_t i = j << (k + 1);
      const uint32_t c = sw[i];
      const uint32_t* op = ops[k];
      sw[i] = op[c & 0xffu] ^ op[256u + ((c >> 8) & 0xffu)] ^ op[512u + ((c >> 16) & 0xffu)] ^
              op[768u + (c >> 24)] ^ sw[i + half];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = ~sw[0];
}

// Many spans at once (launch_span_many): workgroup b folds span b's leaves, parts[b] = {first
// leaf, leaves, tree levels}; the same tree as span_combine_kernel with segments of 2^seg_log2 B.
__global__ __launch_bounds__(1024) void span_combine_many_kernel(const uint32_t* __restrict__ pow2,
                                                                 const uint32_t* __restrict__ leaves,
                                                                 const SpanPart* __restrict__ parts, uint32_t seg_log2,
                                                                 uint32_t* __restrict__ out) {
  __shared__ uint32_t sw[1u << PDB_SPAN_MAX_SEGS_LOG2];
  __shared__ uint32_t ops[PDB_SPAN_MAX_SEGS_LOG2][1024];
  const SpanPart p = parts[blockIdx.x];
  const uint32_t M = 1u << p.m_log2;
  for (uint32_t i = threadIdx.x; i < p.m_log2 * 1024u; i += blockDim.x)
    ops[i >> 10][i & 1023u] = pow2[(seg_log2 + (i >> 10)) * 1024u + (i & 1023u)];
  const uint32_t pad = M - p.nleaves;
  for (uint32_t i = threadIdx.x; i < M; i += blockDim.x) sw[i] = i < pad ? 0u : ~leaves[p.leaf0 + i - pad];
  __syncthreads();
  for (uint32_t k = 0; k < p.m_log2; ++k) {
    const uint32_t half = 1u << k, pairs = M >> (k + 1);
    for (uint32_t j = threadIdx.x; j < pairs; j += blockDim.x) {
      const uint32_t i = j << (k + 1);
      const uint32_t c = sw[i];
      const uint32_t* op = ops[k];
      sw[i] = op[c & 0xffu] ^ op[256u + ((c >> 8) & 0xffu)] ^ op[512u + ((c >> 16) & 0xffu)] ^
              op[768u + (c >> 24)] ^ sw[i + half];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = ~sw[0];
}

// ---- the long-block lane (crc32c_internal.h): pieces, then one combine per record ----------------
// Every piece the batch kernel exported, hashed by the sstable-sized kernel over a piece list (a full
// piece: exactly its 4-KiB body path, started from state 0; a head: Value()'s seed -- the fast path
// at 4096 B, the slow path below), one raw state per piece.  The count is read on the device: the
// launch is made whether or not anything was exported, and returns at once when nothing was.
constexpr uint32_t kPieceWaves = 12;  // (16 waves: 128 VGPRs, 24 of them spilled; 12 as the sstable kernels: 5)
__global__ __launch_bounds__(kPieceWaves * 64) void crc_longpiece_kernel(const uint32_t* __restrict__ tabs, LongLane ll) {
  const uint64_t np = ll.hdr[0] & kLongPieceMask;
  // (a workgroup whose share of the pieces is empty leaves before staging its 160 KiB of tables)
  if (np * blockIdx.x / gridDim.x == np * (blockIdx.x + 1u) / gridDim.x) return;
  sized_kernel_body<PieceSrc, LeafSink, true, 4, false, 4, QuadTabs, false, true, kPieceWaves>(tabs, PieceSrc{ll.piece}, np,
                                                                                              LeafSink{ll.leaf});
}

// op_k(c) through a power-of-two operator (4 x 256 entries) in LDS or global memory
__device__ __forceinline__ uint32_t apply_op(const uint32_t* op, uint32_t c) {
  return op[c & 0xffu] ^ op[256u + ((c >> 8) & 0xffu)] ^ op[512u + ((c >> 16) & 0xffu)] ^ op[768u + (c >> 24)];
}

constexpr uint32_t kCombLog2 = 13;  // leaves folded in LDS at once (2^13 = 32 MiB of block)
constexpr uint32_t kComb = 1u << kCombLog2;

// Workgroup r folds record r's leaves (front-padded with zero leaves to a power of two, or to a
// multiple of 2^13 in chunks, each chunk's root shifted on by 2^13 pieces = 32 MiB), corrects an
// Extend seed (R_s(B) = R_FFFFFFFF(B) ^ shift(s ^ 0xFFFFFFFF, n)), and hands the raw state to the
// batch's sink.  The last workgroup to finish resets the lane's counters for the next call.
constexpr uint32_t kCombThreads = 1024;  // (256: the operators' staging and the first folds 4x longer)
template <class Sink>
__global__ __launch_bounds__(kCombThreads) void long_combine_kernel(LongLane ll, Sink sink) {
  __shared__ uint32_t sw[kComb];
  __shared__ __attribute__((aligned(16))) uint32_t ops[kCombLog2][1024];  // level k: shift 4096 << k (power-of-two operator 12 + k)
  const unsigned long long hw = ll.hdr[0];
  const uint32_t nrec = static_cast<uint32_t>(hw >> 40);
  // Only the min(records, grid) workgroups with a record take part (and count themselves out below):
  // the others leave at once.  One that starts after the reset reads 0 records and leaves too -- every
  // workgroup with a record has counted itself before the reset.
  if (blockIdx.x >= nrec) return;
  const uint32_t t = threadIdx.x;
  {
    uint32_t staged = 0;  // level operators staged so far (grown as records need them: a 64-KiB block needs 5)
    for (uint32_t r = blockIdx.x; r < nrec; r += gridDim.x) {
      const LongRec R = ll.rec[r];
      uint32_t ml = 0;
      while ((1u << ml) < R.np && ml < kCombLog2) ++ml;
      if (ml > staged) {  // (workgroup-uniform; the first barrier below orders it)
        // (16-B loads: levels are 4 KiB, 16-B aligned in the operator table)
        const uint4* src = reinterpret_cast<const uint4*>(ll.pow2 + 12u * 1024u);
        uint4* dst = reinterpret_cast<uint4*>(&ops[0][0]);
        for (uint32_t i = staged * 256u + t; i < ml * 256u; i += blockDim.x) dst[i] = src[i];
        staged = ml;
      }
      const uint32_t M = 1u << ml, nc = (R.np + M - 1u) / M;
      const uint32_t pad = nc * M - R.np;
      uint32_t acc = 0;  // (thread 0)
      for (uint32_t c = 0; c < nc; ++c) {
        __syncthreads();  // the previous fold's root has been read
        for (uint32_t j = t; j < M; j += blockDim.x) {
          const uint32_t v = c * M + j;
          sw[j] = v < pad ? 0u : ll.leaf[R.q0 + (v - pad)];
        }
        __syncthreads();
        for (uint32_t k = 0; k < ml; ++k) {
          const uint32_t half = 1u << k, pairs = M >> (k + 1);
          for (uint32_t j = t; j < pairs; j += blockDim.x) {
            const uint32_t i = j << (k + 1);
            sw[i] = apply_op(ops[k], sw[i]) ^ sw[i + half];
          }
          __syncthreads();
        }
        if (t == 0) acc = c ? apply_op(ll.pow2 + (12u + kCombLog2) * 1024u, acc) ^ sw[0] : sw[0];
      }
      if (t == 0) {
        uint32_t raw = acc;
        if (R.init_raw != 0xFFFFFFFFu) {  // an Extend seed (descriptor batches with PDB_CRC_USE_INIT)
          uint32_t x = R.init_raw ^ 0xFFFFFFFFu;
          for (uint32_t k = 0; k < 32u; ++k)
            if ((R.n >> k) & 1u) x = apply_op(ll.pow2 + k * 1024u, x);
          raw ^= x;
        }
        const BlkDesc d{reinterpret_cast<const uint8_t*>(R.p), R.n, R.init_raw};
        SinkOps<Sink>::put(sink, R.i, raw, d, SinkOps<Sink>::pre(sink, R.i, d));
      }
    }
  }
  __syncthreads();
  if (t == 0) {
    __threadfence();
    if (atomicAdd(ll.hdr + 1, 1ull) + 1ull == (nrec < gridDim.x ? nrec : gridDim.x)) {
      ll.hdr[0] = 0ull;
      ll.hdr[1] = 0ull;
    }
  }
}

// The lane's two launches after a batch kernel with sink `sink` (same stream)
template <class Sink>
hipError_t launch_long(const LaunchGeom& g, const uint32_t* d_tables, const LongLane* ll, const Sink& sink, hipStream_t s) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !ll || !ll->hdr) return e;
  hipLaunchKernelGGL(crc_longpiece_kernel, dim3(g.grid), dim3(kPieceWaves * 64), 0, s, d_tables, *ll);
  hipLaunchKernelGGL((long_combine_kernel<Sink>), dim3(g.grid), dim3(kCombThreads), 0, s, *ll, sink);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_span_many(const LaunchGeom& g, const uint32_t* d_tables, const uint32_t* d_pow2, const uint8_t* base,
                            const pdb_blk* pieces, uint64_t npieces, const SpanPart* parts, uint32_t nparts,
                            uint32_t seg_log2, uint32_t* leaves, uint32_t* out, hipStream_t s) {
  if (nparts == 0) return hipSuccess;
  hipError_t e = launch_desc(g, d_tables, base, pieces, npieces, PDB_CRC_USE_INIT, kModeOut, nullptr, leaves, nullptr,
                             nullptr, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(span_combine_many_kernel, dim3(nparts), dim3(1024), 0, s, d_pow2, leaves, parts, seg_log2, out);
  return hipGetLastError();
}

uint64_t span_scratch_words(uint64_t n, uint32_t min_seg_log2) { return span_geom(n, min_seg_log2).nf + 1; }

hipError_t launch_span(const LaunchGeom& g, const uint32_t* d_tables, const uint32_t* d_pow2,
                       uint32_t init, const uint8_t* data, uint64_t n, uint32_t* scratch, uint32_t* out,
                       hipStream_t s, uint32_t min_seg_log2) {
  const SpanGeom sg = span_geom(n, min_seg_log2);
  // head leaf from the Extend seed (n mod S bytes, possibly empty), then the full segments
  hipError_t e = launch_fixed(g, d_tables, data, 0, static_cast<uint32_t>(sg.head), 1, PDB_CRC_USE_INIT,
                              init, scratch, s);
  if (e != hipSuccess) return e;
  if (sg.nf) {
    const uint64_t S = 1ull << sg.seg_log2;
    e = launch_fixed(g, d_tables, data + sg.head, S, static_cast<uint32_t>(S), sg.nf, PDB_CRC_USE_INIT,
                     0xFFFFFFFFu, scratch + 1, s);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(span_combine_kernel, dim3(1), dim3(1024), 0, s, d_pow2, scratch, sg.seg_log2,
                     sg.m_log2, sg.nf + 1, out);
  return hipGetLastError();
}

hipError_t launch_fixed(const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                        uint64_t stride, uint32_t len, uint64_t nblk, uint32_t flags, uint32_t init,
                        uint32_t* out, hipStream_t s) {
  if (nblk == 0) return hipSuccess;
  const dim3 grid(grid_for(g, nblk)), block(kThreads);
  const bool fast = len == 4096u && (reinterpret_cast<uintptr_t>(base) & 15u) == 0 && (stride & 15u) == 0;
  if (fast) {
    // 4 blocks per wave-iteration, one packed tree, workgroup lock-step per 4-block group; lane
    // pieces 4 x 16 B so every load instruction reads 1 KiB contiguous, with the nt policy
    // (A/B: profiles/r01_ab_pack4k_nt*.json, +7-10 % over 2 x 32-B pieces with default loads)
    hipLaunchKernelGGL(crc_pack4k_kernel<>, grid, block, 0, s, d_tables, base, stride, nblk, flags, init, out);
    return hipGetLastError();
  }
  const FixedSrc src{base, stride, len, (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu};
  const OutSink sink{out, flags};
  if (src.init_raw == 0xFFFFFFFFu) {
    // Value()-seeded size classes (the same kernels as the descriptor hints; tests/test_sst4k.py
    // covers fixed strides of every class at every alignment)
    if (len - kSstMin <= kSstMax - kSstMin) {
      // sstable-sized blocks (4096..4352 B, any alignment): exact 4-KiB body + batched prefix
      // (profiles/r01_ab_sst4k.json)
      // (12 waves: fewer spills, +1.3 % in A/B, profiles/r03_waves/ab_waves2.log; diagnostics 130)
      hipLaunchKernelGGL((crc_sst4k_kernel<FixedSrc, OutSink, true, 4, QuadTabs, false, true, 12>), grid, dim3(768), 0, s,
                         d_tables, src, nblk, sink);
      return hipGetLastError();
    }
    if (len - 1u <= 1151u) {  // records of 1..1152 B, staged through LDS, k lanes each (crc32c_lanespan.h)
      return launch_lanespan(g, d_tables, src, nblk,
                             len <= 256u ? 256u : (len <= 512u ? 512u : (len <= 1023u ? 1023u : 1152u)), sink, s);
    }
  }
  // any other length / seed: stream kernels with workgroup-local dynamic blocks and packed 4-block
  // trees.  4-B-aligned pieces: 16-B lane pieces with nt loads; otherwise 32-B pieces (per-block
  // misalignment makes the 16-B kernel's neighbour-dword path cost more than nt gains: sstable
  // layout 6.1 vs 5.8 TB/s, profiles/r01_ab_gen_pack.json)
  const bool aligned4 = ((reinterpret_cast<uintptr_t>(base) + (len & 15u)) & 3u) == 0 && (stride & 3u) == 0;
  if (aligned4)
    hipLaunchKernelGGL((crc_stream16_kernel<FixedSrc, OutSink, true, true, true>), grid, block, 0, s, d_tables, src,
                       nblk, sink);
  else
    hipLaunchKernelGGL((crc_stream_kernel<FixedSrc, OutSink, 0, true, true>), grid, block, 0, s, d_tables, src, nblk,
                       sink);
  return hipGetLastError();
}

namespace {

// Descriptor batches: the size-class hint picks the kernel (speed only; Value() seeds only, an
// Extend seed takes the any-length kernel).  Other lengths inside a hinted batch take each
// kernel's own slow path in the same launch.
template <class Sink>
hipError_t launch_desc_sink(const LaunchGeom& g, const uint32_t* d_tables, const DescSrc& src, uint64_t nblk,
                            uint32_t flags, const Sink& sink, hipStream_t s) {
  const dim3 grid(grid_for(g, nblk)), block(kThreads);
  const uint32_t hint =
      flags & (PDB_CRC_SIZE_1K | PDB_CRC_SIZE_4K | PDB_CRC_SIZE_256 | PDB_CRC_SIZE_512 | PDB_CRC_SIZE_1023);
  if (hint && !(flags & PDB_CRC_USE_INIT)) {
    if (flags & PDB_CRC_SIZE_1K)  // WAL records of ~1-KiB batches: the record kernel's 1152 class
      // (+4-6 % over crc_sst1k_kernel's 8-block groups, profiles/r02_wal1k/; diagnostics variant 68)
      return launch_lanespan(g, d_tables, src, nblk, 1152u, sink, s);
    if (flags & PDB_CRC_SIZE_4K) {  // sstable data blocks: 4-KiB body + batched prefix
      hipLaunchKernelGGL((crc_sst4k_kernel<DescSrc, Sink, true>), grid, block, 0, s, d_tables, src, nblk, sink);
      return hipGetLastError();
    }
    // records of 1..1023 B: k lanes per record, the bytes staged through LDS by coalesced loads
    return launch_lanespan(g, d_tables, src, nblk,
                           (flags & PDB_CRC_SIZE_256) ? 256u : ((flags & PDB_CRC_SIZE_512) ? 512u : 1023u), sink, s,
                           (flags & PDB_CRC_SIZE_MIXED) != 0);
  }
  // descriptor lists of any lengths (C3: Zipf sizes at byte offsets): 16-B lane pieces with nt
  // loads, dynamic blocks, packed 4-block trees (A/B: profiles/r01_ab_c3_pack*.json), byte-balanced
  // workgroup ranges (bal_bound; diagnostics variant 71 splits by block count)
  hipLaunchKernelGGL((crc_stream16_kernel<DescSrc, Sink, true, true, true, QuadTabs, true>), grid, block, 0, s,
                     d_tables, src, nblk, sink);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_desc(const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                       const pdb_blk* blk, uint64_t nblk, uint32_t flags, int mode,
                       const uint32_t* expected, uint32_t* out, uint8_t* ok, uint32_t* nbad,
                       hipStream_t s, const LongLane* ll) {
  if (nblk == 0) return hipSuccess;
  // small-record hints (WAL / MANIFEST records: physical records are <= 32 KiB, log_format.h:24-33)
  // take no long-block lane: its two launches would cost those batches 1-2 % (tools/ab_lane.sh), and
  // a record outside the class is hashed by the record kernel's whole-wave path
  const bool small = (flags & (PDB_CRC_SIZE_1K | PDB_CRC_SIZE_256 | PDB_CRC_SIZE_512 | PDB_CRC_SIZE_1023)) &&
                     !(flags & (PDB_CRC_USE_INIT | PDB_CRC_SIZE_4K));
  if (small) ll = nullptr;
  DescSrc src{base, blk, flags};
  if (ll) src.long_lane = reinterpret_cast<uint8_t*>(ll->hdr);
  if (mode == kModeOut) {
    const OutSink sink{out, flags};
    (void)launch_desc_sink(g, d_tables, src, nblk, flags, sink, s);
    return launch_long(g, d_tables, ll, sink, s);
  }
  const VerifySink sink{expected, ok, nbad, flags};
  (void)launch_desc_sink(g, d_tables, src, nblk, flags, sink, s);
  return launch_long(g, d_tables, ll, sink, s);
}

hipError_t launch_sst(const LaunchGeom& g, const uint32_t* d_tables, uint8_t* buf, uint64_t buf_len,
                      const pdb_block_handle* h, uint64_t n, bool seal, uint8_t* ok, uint32_t* nbad,
                      hipStream_t s, const LongLane* ll) {
  if (n == 0) return hipSuccess;
  const dim3 grid(grid_for(g, n));
  // exact 4-KiB body + batched prefix for the 4096..4352-B blocks (every data block TableBuilder
  // emits: contents + type), the slow path in the same launch for the rest, and the long-block lane
  // for blocks of >= 16 KiB (a table's index and filter blocks)
  // (profiles/r01_ab_sst4k.json: verify +45 %, seal +27 % over crc_stream16_kernel)
  SstSrc src{buf, h, buf_len};  // handles outside the image are reported, never followed
  if (ll) src.long_lane = reinterpret_cast<uint8_t*>(ll->hdr);
  // seal: each wave parks its trailers (4 per lane) and writes them 64 groups later or when it is
  // done -- writing a trailer soon after its line was read costs more (DESIGN.md §6.0, f2:
  // +4.8 % over writing each group's trailers when hashed; diagnostics variant 72 is that form).
  // 12 waves (168 VGPRs a lane: 10 spills instead of 44-53 at 16 waves): +2.5 % over round 5's
  // 16-wave seal, both orders on one box (tools/ab_lane.sh, profiles/r06/ab_lane/ab_seal.log)
  if (seal) {
    hipLaunchKernelGGL((crc_sst4k_kernel<SstSrc, ParkSealSink<64>, true, 4, QuadTabs, false, true, 12>), grid, dim3(768), 0,
                       s, d_tables, src, n, ParkSealSink<64>{});
    return launch_long(g, d_tables, ll, ParkSealSink<64>{}, s);
  }
  // verify: 12 waves (168 VGPRs a lane: 32 B of spills instead of 124 at 16 waves), +1.2-1.7 % in
  // A/B both orders (profiles/r03_waves/; diagnostics 127 / 128 / 129 = 12 / 8 / 16 waves)
  hipLaunchKernelGGL((crc_sst4k_kernel<SstSrc, SstVerifySink, true, 4, QuadTabs, false, true, 12>), grid, dim3(768), 0,
                     s, d_tables, src, n, SstVerifySink{ok, nbad});
  return launch_long(g, d_tables, ll, SstVerifySink{ok, nbad}, s);
}

hipError_t launch_sst_masked(const LaunchGeom& g, const uint32_t* d_tables, uint8_t* buf, uint64_t buf_len,
                             const pdb_block_handle* h, uint64_t n, uint32_t* out, hipStream_t s, const LongLane* ll) {
  if (n == 0) return hipSuccess;
  // the seal's masked CRCs into a compact array (pdb_sst_crc_device; the host seal brings back 4 B
  // per block across PCIe, not the span)
  SstSrc src{buf, h, buf_len};
  if (ll) src.long_lane = reinterpret_cast<uint8_t*>(ll->hdr);
  // (12 waves: fewer spills, +0.7 % in A/B, profiles/r03_waves/ab_waves2.log; diagnostics 131 / 132)
  hipLaunchKernelGGL((crc_sst4k_kernel<SstSrc, SstCrcSink, true, 4, QuadTabs, false, true, 12>), dim3(grid_for(g, n)),
                     dim3(768), 0, s, d_tables, src, n, SstCrcSink{out});
  return launch_long(g, d_tables, ll, SstCrcSink{out}, s);
}

}  // namespace pdb
