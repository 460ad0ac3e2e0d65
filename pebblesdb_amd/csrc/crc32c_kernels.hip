// crc32c_kernels.hip -- CRC32C (Castagnoli) over batches of independent sstable blocks on
// MI355X (gfx950, CDNA4).  Hand-written HIP; no MFMA (GF(2) byte work is not a contraction).
//
// Replaces the per-block software CRC of the reference: crc32c::Extend -> crc32_software ->
// crc32c_sb8_64_bit (util/crc32c.cc:25-32, 101-103, 585-625), called once per block by
// TableBuilder::WriteRawBlock (table/table_builder.cc:197-199) and ReadBlock
// (table/format.cc:96-98).  Results are bit-identical (tests/golden + oracle parity).
//
// Shipped launches (the kernels themselves live in crc32c_device.h):
//   * crc_pack4k_kernel<1, 4, nt> -- fixed stride, 4-KiB, 16-B aligned blocks (BASELINE configs
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
// LDS image (crc32c_math.h): T0..T3 replicated 32x (128 KiB) so each lane reads its own bank +
// 8 shift-operator slots (32 KiB): the whole 160 KiB of a CU; one 1024-thread workgroup per CU
// stages it once and walks blocks persistently.  DESIGN.md §3-§6 has the measurements.
#include "crc32c_device.h"

namespace pdb {
namespace {

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

__host__ __device__ inline SpanGeom span_geom(uint64_t n) {
  SpanGeom g;
  g.seg_log2 = PDB_SPAN_MIN_SEG_LOG2;
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

}  // namespace

int g_fast_variant = 0;  // diagnostics: pdb_diag_set_variant()

uint64_t span_scratch_words(uint64_t n) { return span_geom(n).nf + 1; }

hipError_t launch_span(const LaunchGeom& g, const uint32_t* d_tables, const uint32_t* d_pow2,
                       uint32_t init, const uint8_t* data, uint64_t n, uint32_t* scratch, uint32_t* out,
                       hipStream_t s) {
  const SpanGeom sg = span_geom(n);
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
  if (g_fast_variant != 0)
    return launch_fixed_variant(g_fast_variant, g, d_tables, base, stride, len, nblk, flags, init, out, s);
  const dim3 grid(grid_for(g, nblk)), block(kThreads);
  const bool fast = len == 4096u && (reinterpret_cast<uintptr_t>(base) & 15u) == 0 &&
                    (stride & 15u) == 0;
  if (fast) {
    // 4 blocks per wave-iteration, one packed tree, workgroup lock-step per 4-block group; lane
    // pieces 4 x 16 B so every load instruction reads 1 KiB contiguous, with the nt policy
    // (A/B: profiles/r01_ab_pack4k_nt*.json, +7-10 % over 2 x 32-B pieces with default loads)
    hipLaunchKernelGGL((crc_pack4k_kernel<1, 4, true>), grid, block, 0, s, d_tables, base, stride, nblk, flags,
                       init, out);
  } else {
    // any length / alignment: stream kernels with workgroup-local dynamic blocks and packed
    // 4-block trees.  4-B-aligned pieces: 16-B lane pieces with nt loads; otherwise 32-B pieces
    // (per-block misalignment makes the 16-B kernel's neighbour-dword path cost more than nt
    // gains: sstable layout 6.1 vs 5.8 TB/s, profiles/r01_ab_gen_pack.json)
    const FixedSrc src{base, stride, len, (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu};
    if (len - kSstMin <= kSstMax - kSstMin && src.init_raw == 0xFFFFFFFFu) {
      // sstable-sized blocks (4096..4352 B, any alignment, Value() seed): exact 4-KiB body +
      // batched prefix (profiles/r01_ab_sst4k.json)
      hipLaunchKernelGGL((crc_sst4k_kernel<FixedSrc, OutSink, true>), grid, block, 0, s, d_tables, src, nblk,
                         OutSink{out, flags});
      return hipGetLastError();
    }
    if (src.init_raw == 0xFFFFFFFFu && (len - 1024u <= 128u || len - 1u <= 1022u)) {
      // the same size classes as the descriptor hints: 1-KiB records (1024..1152 B) and records
      // of 1..256 B (tests/test_sst4k.py: fixed strides at every alignment)
      if (len >= 1024u)
        hipLaunchKernelGGL((crc_sst1k_kernel<FixedSrc, OutSink, true>), grid, block, 0, s, d_tables, src, nblk,
                           OutSink{out, flags});
      else if (len <= 256u)  // one lane per record (profiles/r01_ab_lanerec.json)
        hipLaunchKernelGGL((crc_lanerec9_kernel<FixedSrc, OutSink>), dim3(grid_for(g, (nblk + 63) / 64)), block, 0,
                           s, d_tables, src, nblk, OutSink{out, flags});
      else if (len > 512u)  // 513..1023 B: the 33-group window
        hipLaunchKernelGGL((crc_lanerec33_kernel<FixedSrc, OutSink>), dim3(grid_wg(g, nblk, 256)), dim3(256), 0, s,
                           d_tables, src, nblk, OutSink{out, flags});
      else  // 257..512 B: the 17-group window
        hipLaunchKernelGGL((crc_lanerec17_kernel<FixedSrc, OutSink>), dim3(grid17(g, nblk)), dim3(kThreads17), 0,
                           s, d_tables, src, nblk, OutSink{out, flags});
      return hipGetLastError();
    }
    const bool aligned4 = ((reinterpret_cast<uintptr_t>(base) + (len & 15u)) & 3u) == 0 && (stride & 3u) == 0;
    if (aligned4)
      hipLaunchKernelGGL((crc_stream16_kernel<FixedSrc, OutSink, true, true, true>), grid, block, 0, s, d_tables,
                         src, nblk, OutSink{out, flags});
    else
      hipLaunchKernelGGL((crc_stream_kernel<FixedSrc, OutSink, 0, true, true>), grid, block, 0, s, d_tables, src,
                         nblk, OutSink{out, flags});
  }
  return hipGetLastError();
}

hipError_t launch_desc(const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                       const pdb_blk* blk, uint64_t nblk, uint32_t flags, int mode,
                       const uint32_t* expected, uint32_t* out, uint8_t* ok, uint32_t* nbad,
                       hipStream_t s) {
  if (nblk == 0) return hipSuccess;
  // 40: ignore size hints; 41: the 1-KiB kernel with 4-block groups; 50/51: one lane per record
  // with 32-B groups loaded one ahead (nt / default loads), 52: the shipped fixed-window version,
  // for any list; 53: the <= 256-B class on the previous crc_rec256_kernel
  if (g_fast_variant >= 50 && g_fast_variant <= 52 && !(flags & PDB_CRC_USE_INIT)) {
    const dim3 grid(grid_for(g, (nblk + 63) / 64)), block(kThreads);
    const DescSrc src{base, blk, flags};
    if (mode == kModeOut && g_fast_variant == 52)
      hipLaunchKernelGGL((crc_lanerec9_kernel<DescSrc, OutSink>), grid, block, 0, s, d_tables, src, nblk,
                         OutSink{out, flags});
    else if (mode == kModeOut) {
      if (g_fast_variant == 50)
        hipLaunchKernelGGL((crc_lanerec_kernel<DescSrc, OutSink, true>), grid, block, 0, s, d_tables, src, nblk,
                           OutSink{out, flags});
      else
        hipLaunchKernelGGL((crc_lanerec_kernel<DescSrc, OutSink, false>), grid, block, 0, s, d_tables, src, nblk,
                           OutSink{out, flags});
    } else {
      hipLaunchKernelGGL((crc_lanerec9_kernel<DescSrc, VerifySink>), grid, block, 0, s, d_tables, src, nblk,
                         VerifySink{expected, ok, nbad, flags});
    }
    return hipGetLastError();
  }
  if (mode == kModeOut && g_fast_variant != 0 && g_fast_variant != 40 && g_fast_variant != 41 && g_fast_variant != 53 &&
      (g_fast_variant < 54 || g_fast_variant > 58))
    return launch_desc_variant(g_fast_variant, g, d_tables, base, blk, nblk, flags, out, s);
  const dim3 grid(grid_for(g, nblk)), block(kThreads);
  const DescSrc src{base, blk, flags};
  // size-class hints (Value() seeds only): the sized kernels (exact 1-/4-KiB body + batched
  // prefix; other lengths take their slow path in the same launch)
  if (!(flags & PDB_CRC_USE_INIT) && (flags & (PDB_CRC_SIZE_1K | PDB_CRC_SIZE_4K | PDB_CRC_SIZE_256 | PDB_CRC_SIZE_512 | PDB_CRC_SIZE_1023)) &&
      g_fast_variant != 40) {
    const bool k1 = flags & PDB_CRC_SIZE_1K;
    if (!k1 && !(flags & PDB_CRC_SIZE_4K)) {
      // records <= 256 B: one lane per record on a fixed 288-B window, all loads up front, two
      // chains (wal100 1387 -> 3485 GB/s, 256-B records 2507 -> 3835 GB/s over the rows-of-16-lanes
      // crc_rec256_kernel, A/B variant 53: profiles/r01_ab_lanerec.json); other lengths take the
      // whole-wave slow path in the same launch
      const dim3 lgrid(grid_for(g, (nblk + 63) / 64));
      if (!(flags & (PDB_CRC_SIZE_256 | PDB_CRC_SIZE_512)) && g_fast_variant != 40) {
        // 513..1023-B class: the 33-group (1056-B) window, 8 chains, 256-thread workgroups (one wave
        // per SIMD; the window spills into AGPRs, not scratch): 1.33x the generic kernel on 700-B
        // records, 1.03-1.07x on uniform 513..1024 B (profiles/r01_ab_rec1023.json)
        const dim3 g33(grid_wg(g, nblk, 256));
        if (mode == kModeOut)
          hipLaunchKernelGGL((crc_lanerec33_kernel<DescSrc, OutSink>), g33, dim3(256), 0, s, d_tables, src, nblk,
                             OutSink{out, flags});
        else
          hipLaunchKernelGGL((crc_lanerec33_kernel<DescSrc, VerifySink>), g33, dim3(256), 0, s, d_tables, src, nblk,
                             VerifySink{expected, ok, nbad, flags});
        return hipGetLastError();
      }
      if (!(flags & PDB_CRC_SIZE_256)) {
        // 257..512-B class: the same lane-per-record design on a 17-group (544-B) window, chains
        // of 9 + 8 groups; records of 1..512 B all take the fast path
        if (mode == kModeOut && g_fast_variant == 58)  // A/B: four lanes per record
          hipLaunchKernelGGL((crc_quadrec_kernel<DescSrc, OutSink, 9, 512>), dim3(grid_for(g, (nblk + 15) / 16)), block,
                             0, s, d_tables, src, nblk, OutSink{out, flags});
        else if (mode == kModeOut && g_fast_variant == 56)  // A/B: cross-batch prefetch, 256 threads
          hipLaunchKernelGGL((crc_lanerec_pf_kernel<DescSrc, OutSink, 17, 256>), dim3(grid_wg(g, nblk, 256)),
                             dim3(256), 0, s, d_tables, src, nblk, OutSink{out, flags});
        else if (mode == kModeOut && g_fast_variant == 54)  // A/B: two chains (9 + 8 groups)
          hipLaunchKernelGGL((crc_lanerec17_kernel<DescSrc, OutSink, 2>), dim3(grid17(g, nblk)), dim3(kThreads17), 0,
                             s, d_tables, src, nblk, OutSink{out, flags});
        else if (mode == kModeOut)
          hipLaunchKernelGGL((crc_lanerec17_kernel<DescSrc, OutSink>), dim3(grid17(g, nblk)), dim3(kThreads17), 0, s,
                             d_tables, src, nblk, OutSink{out, flags});
        else
          hipLaunchKernelGGL((crc_lanerec17_kernel<DescSrc, VerifySink>), dim3(grid17(g, nblk)), dim3(kThreads17), 0,
                             s, d_tables, src, nblk, VerifySink{expected, ok, nbad, flags});
        return hipGetLastError();
      }
      if (mode == kModeOut && g_fast_variant == 57)  // A/B: four lanes per record
        hipLaunchKernelGGL((crc_quadrec_kernel<DescSrc, OutSink, 5, 256>), dim3(grid_for(g, (nblk + 15) / 16)), block,
                           0, s, d_tables, src, nblk, OutSink{out, flags});
      else if (mode == kModeOut && g_fast_variant == 55)  // A/B: cross-batch prefetch, 512 threads
        hipLaunchKernelGGL((crc_lanerec_pf_kernel<DescSrc, OutSink, 9, 512>), dim3(grid_wg(g, nblk, 512)),
                           dim3(512), 0, s, d_tables, src, nblk, OutSink{out, flags});
      else if (mode == kModeOut && g_fast_variant == 53)
        hipLaunchKernelGGL((crc_rec256_kernel<DescSrc, OutSink, true>), grid, block, 0, s, d_tables, src, nblk,
                           OutSink{out, flags});
      else if (mode == kModeOut)
        hipLaunchKernelGGL((crc_lanerec9_kernel<DescSrc, OutSink>), lgrid, block, 0, s, d_tables, src, nblk,
                           OutSink{out, flags});
      else
        hipLaunchKernelGGL((crc_lanerec9_kernel<DescSrc, VerifySink>), lgrid, block, 0, s, d_tables, src, nblk,
                           VerifySink{expected, ok, nbad, flags});
      return hipGetLastError();
    }
#define PDB_SIZED(K, SINK, ...)                                                                                   \
  hipLaunchKernelGGL((K<DescSrc, SINK, true>), grid, block, 0, s, d_tables, src, nblk, SINK{__VA_ARGS__})
#define PDB_SIZED1K4(SINK, ...)                                                                                  \
  hipLaunchKernelGGL((crc_sst1k_kernel<DescSrc, SINK, true, 4>), grid, block, 0, s, d_tables, src, nblk,         \
                     SINK{__VA_ARGS__})
    // 1-KiB class: 8-block groups (fast range 1024..1152 B: WAL records of ~1-KiB batches), A/B
    // variant 41 the 4-block version (1024..1280 B)
    const bool g4 = g_fast_variant == 41;
    if (mode == kModeOut) {
      if (k1 && g4) PDB_SIZED1K4(OutSink, out, flags);
      else if (k1) PDB_SIZED(crc_sst1k_kernel, OutSink, out, flags);
      else PDB_SIZED(crc_sst4k_kernel, OutSink, out, flags);
    } else {
      if (k1 && g4) PDB_SIZED1K4(VerifySink, expected, ok, nbad, flags);
      else if (k1) PDB_SIZED(crc_sst1k_kernel, VerifySink, expected, ok, nbad, flags);
      else PDB_SIZED(crc_sst4k_kernel, VerifySink, expected, ok, nbad, flags);
    }
#undef PDB_SIZED1K4
#undef PDB_SIZED
    return hipGetLastError();
  }
  // descriptor lists (C3: Zipf sizes at byte offsets): 16-B lane pieces with nt loads, dynamic
  // blocks, packed 4-block trees (A/B: profiles/r01_ab_c3_pack*.json)
  if (mode == kModeOut)
    hipLaunchKernelGGL((crc_stream16_kernel<DescSrc, OutSink, true, true, true>), grid, block, 0, s, d_tables,
                       src, nblk, OutSink{out, flags});
  else
    hipLaunchKernelGGL((crc_stream16_kernel<DescSrc, VerifySink, true, true, true>), grid, block, 0, s, d_tables,
                       src, nblk, VerifySink{expected, ok, nbad, flags});
  return hipGetLastError();
}


hipError_t launch_sst(const LaunchGeom& g, const uint32_t* d_tables, uint8_t* buf, uint64_t buf_len,
                      const pdb_block_handle* h, uint64_t n, bool seal, uint8_t* ok, uint32_t* nbad,
                      hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (g_fast_variant != 0) return launch_sst_variant(g_fast_variant, g, d_tables, buf, buf_len, h, n, seal, ok, nbad, s);
  const dim3 grid(grid_for(g, n)), block(kThreads);
  // exact 4-KiB body + batched prefix for the 4096..4352-B blocks (every data block TableBuilder
  // emits: contents + type), the slow path in the same launch for the rest
  // (profiles/r01_ab_sst4k.json: verify +45 %, seal +27 % over crc_stream16_kernel)
  const SstSrc src{buf, h, buf_len};  // handles outside the image are reported, never followed
  if (seal)
    hipLaunchKernelGGL((crc_sst4k_kernel<SstSrc, SealSink, true>), grid, block, 0, s, d_tables, src, n, SealSink{});
  else
    hipLaunchKernelGGL((crc_sst4k_kernel<SstSrc, SstVerifySink, true>), grid, block, 0, s, d_tables, src, n,
                       SstVerifySink{ok, nbad});
  return hipGetLastError();
}

hipError_t launch_sst_masked(const LaunchGeom& g, const uint32_t* d_tables, uint8_t* buf, uint64_t buf_len,
                             const pdb_block_handle* h, uint64_t n, uint32_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const dim3 grid(grid_for(g, n)), block(kThreads);
  // the seal's masked CRCs into a compact array (pdb_sst_crc_device; the host seal brings back 4 B
  // per block across PCIe, not the span)
  const SstSrc src{buf, h, buf_len};
  if (g_fast_variant == 0)
    hipLaunchKernelGGL((crc_sst4k_kernel<SstSrc, SstCrcSink, true>), grid, block, 0, s, d_tables, src, n,
                       SstCrcSink{out});
  else
    hipLaunchKernelGGL((crc_stream16_kernel<SstSrc, SstCrcSink, true, true, true>), grid, block, 0, s, d_tables, src,
                       n, SstCrcSink{out});
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
