// diag_variants.hip -- BENCH / TEST INFRASTRUCTURE (libpdb_crc32c_diag.so, never linked into the
// product): the synthetic-input fill, the load-pattern calibration kernels behind the roofline and
// pattern-ceiling numbers, the record kernel's part / clock / work-distribution
// diagnostics, and the few alternative kernels the parity tests use as independent cross-checks of
// the product's routing.  Selected per call through include/pdb_crc32c_diag.h.  (The round-1..4
// A/B variants that lost are recorded in DESIGN.md's appendix; round 5 removed them.)
#include "crc32c_device.h"
#include "crc32c_lanespan.h"
#include "diag_internal.h"

namespace pdb {
namespace {

// variants 180-182: the record kernel with per-wave clock stamps, stored after the CRCs in `out`
struct StampOutSink : OutSink {
  uint64_t* stamps;
};

__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Thread t writes dst[8t .. 8t+8) (bytes of the splitmix stream at byte_offset + 8t + j).
__global__ __launch_bounds__(256) void fill_splitmix_kernel(uint8_t* __restrict__ dst, uint64_t nbytes, uint64_t seed,
                                                            uint64_t byte_offset) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint32_t sh = static_cast<uint32_t>(byte_offset & 7u);
  for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t * 8 < nbytes; t += stride) {
    const uint64_t gb = byte_offset + t * 8;  // first global byte of this thread
    const uint64_t w0 = splitmix64_at(seed, gb >> 3);
    uint64_t v = w0;
    if (sh) {
      const uint64_t w1 = splitmix64_at(seed, (gb >> 3) + 1);
      v = (w0 >> (8 * sh)) | (w1 << (64 - 8 * sh));
    }
    if (t * 8 + 8 <= nbytes && (reinterpret_cast<uintptr_t>(dst) & 7u) == 0) {
      *reinterpret_cast<uint64_t*>(dst + t * 8) = v;
    } else {
      for (uint32_t j = 0; j < 8 && t * 8 + j < nbytes; ++j) dst[t * 8 + j] = static_cast<uint8_t>(v >> (8 * j));
    }
  }
}

// ---- load-pattern calibration ------------------------------------------------------------------
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

// The 4-KiB path's loads with no CRC work (pdb_diag_read_pattern4k variant 21, the only one kept):
// lane l reads 16 B at 16 l + 1024 j, j = 0..3 (each load instruction 1 KiB contiguous, nt policy),
// one block per wave at a time, blocks wave-interleaved, every 16 waves of a workgroup in lock-step
// (one __syncthreads per block step).  Also the FETCH_SIZE calibration kernel of tools/pmc_traffic.py.
__global__ __launch_bounds__(kThreads) void read_pattern4k_kernel(const uint8_t* __restrict__ base, uint64_t nblk,
                                                                  uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerWg;
  uint32_t acc = 0;
  const uint64_t first = static_cast<uint64_t>(blockIdx.x) * kWavesPerWg + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t wg_first = static_cast<uint64_t>(blockIdx.x) * kWavesPerWg;
  for (uint64_t b = first, bw = wg_first; bw < nblk; b += nw, bw += nw) {
    __syncthreads();
    u32x4 x = {0, 0, 0, 0};
    if (b < nblk) {
      const uint8_t* blk = base + b * 4096u;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        x ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(blk + lane * 16u + j * 1024u));
    }
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  for (int k = 32; k; k >>= 1) acc ^= __shfl_xor(acc, k, 64);
  if (lane == 0) atomicXor(out, acc);
}

// Seal-pattern calibration (sst variants 140 / 141; no CRC work, trailers written with WRONG values
// by design): the in-place seal's memory pattern without its hash -- every block's bytes [offset,
// offset + size + 5) read as 1-KiB-contiguous 16-B nt loads by the wave owning its 4-block group,
// groups in workgroup lock-step over the workgroup's contiguous range (the sst kernel's
// scheduling), handles a group ahead -- with kWrite 0: no stores (the pattern's read ceiling);
// 1: each group's 4 trailers stored (4 byte stores, like SealSink) once its loads returned;
// 2 / 3 (variants 142 / 143): instead of the 4 trailer bytes, the whole aligned 64-B / 128-B line
// holding them, as 16-B stores (what a seal that rewrote the trailer's line with the bytes it read
// would write: full-line writes, no partial-line merge at the memory side; lines past the image's
// end are skipped).
template <int kWrite>
__global__ __launch_bounds__(kThreads) void seal_pattern_kernel(uint8_t* __restrict__ buf,
                                                                const pdb_block_handle* __restrict__ h,
                                                                uint64_t n, uint32_t* __restrict__ out,
                                                                uint64_t len = 0) {
  typedef __attribute__((address_space(1))) uint8_t g_u8;
  const uint32_t u = threadIdx.x & 63u;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t G = gridDim.x;
  const uint64_t lo = n * blockIdx.x / G, hi = n * (blockIdx.x + 1) / G;
  if (lo >= hi) return;
  uint32_t acc = 0;
  auto hload = [&](uint64_t b0) -> u32x4 {  // lane r < 4: block b0 + r's handle (clamped)
    const uint64_t b = b0 + (u & 3u);
    return gload128<false>(reinterpret_cast<uintptr_t>(h + (b < hi ? b : hi - 1)));
  };
  u32x4 hn = hload(lo + 4u * w);
  for (uint64_t t = 0; lo + 64u * t < hi; ++t) {
    __syncthreads();
    const uint64_t b0 = lo + 4u * (16u * t + w);
    const u32x4 hc = hn;
    keep_alive(hc);
    hn = hload(b0 + 64u);
    u32x4 x = {0, 0, 0, 0};
    uintptr_t ta = 0;  // lane r < 4: block r's trailer word address
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) {
      const uint64_t off = uniform64(__builtin_amdgcn_readlane(hc.x, r), __builtin_amdgcn_readlane(hc.y, r));
      const uint32_t sz = __builtin_amdgcn_readlane(hc.z, r);
      const uintptr_t a0 = (reinterpret_cast<uintptr_t>(buf) + off) & ~static_cast<uintptr_t>(15);
      const uintptr_t e = reinterpret_cast<uintptr_t>(buf) + off + sz + 5u;
      const uint32_t last = static_cast<uint32_t>((e - 1u - a0) >> 4);
#pragma unroll
      for (uint32_t j = 0; j < 5; ++j) {
        const uint32_t c = 64u * j + u;
        x ^= gload128<true>(a0 + 16u * (c < last ? c : last));
      }
      if (u == r) ta = reinterpret_cast<uintptr_t>(buf) + off + sz + 1u;
    }
    const uint32_t m = x.x ^ x.y ^ x.z ^ x.w;
    acc ^= m;
    if constexpr (kWrite == 1) {
      if (u < 4u && b0 + u < hi) {
        g_u8* tr = reinterpret_cast<g_u8*>(ta);
#pragma unroll
        for (int k = 0; k < 4; ++k) tr[k] = static_cast<uint8_t>(m >> (8 * k));
      }
    }
    if constexpr (kWrite >= 2) {
      constexpr uint32_t kLine = kWrite == 2 ? 64u : 128u, kPer = kLine / 16u;
      const uint32_t r = u / kPer, k = u % kPer;
      const uint32_t tl = __shfl(static_cast<uint32_t>(ta), r & 3u, 64), th = __shfl(static_cast<uint32_t>(ta >> 32), r & 3u, 64);
      const uintptr_t base = ((static_cast<uintptr_t>(th) << 32) | tl) & ~static_cast<uintptr_t>(kLine - 1u);
      if (r < 4u && b0 + r < hi && base + kLine <= reinterpret_cast<uintptr_t>(buf) + len)
        *reinterpret_cast<u32x4*>(base + 16u * k) = x;
    }
  }
  for (int k = 32; k; k >>= 1) acc ^= __shfl_xor(acc, k, 64);
  if (u == 0 && out) atomicXor(out, acc);
}

uint32_t record_class(uint32_t flags) {
  return (flags & PDB_CRC_SIZE_256) ? 256u : (flags & PDB_CRC_SIZE_512) ? 512u : ((flags & PDB_CRC_SIZE_1K) ? 1152u : 1023u);
}

}  // namespace

hipError_t launch_sst_variant(int v, const LaunchGeom& g, const uint32_t* d_tables, uint8_t* buf, uint64_t buf_len,
                              const pdb_block_handle* h, uint64_t n, bool seal, uint8_t* ok, uint32_t* nbad,
                              hipStream_t s) {
  const dim3 grid(grid_for(g, n)), block(kThreads);
  const SstSrc src{buf, h, buf_len};
  switch (v) {
    case 140:  // the seal's loads alone / loads + its in-place trailer stores (pattern ceilings;
    case 141:  // wrong trailers by design; nbad = XOR of what was read)
    case 142:  // loads + the 64-B / 128-B line holding each trailer stored whole (wrong bytes there too)
    case 143:
      if (!seal) return hipErrorInvalidValue;
      if (v == 140) hipLaunchKernelGGL(seal_pattern_kernel<0>, grid, block, 0, s, buf, h, n, nbad, buf_len);
      else if (v == 141) hipLaunchKernelGGL(seal_pattern_kernel<1>, grid, block, 0, s, buf, h, n, nbad, buf_len);
      else if (v == 142) hipLaunchKernelGGL(seal_pattern_kernel<2>, grid, block, 0, s, buf, h, n, nbad, buf_len);
      else hipLaunchKernelGGL(seal_pattern_kernel<3>, grid, block, 0, s, buf, h, n, nbad, buf_len);
      return hipGetLastError();
    case 72:  // the seal with each group's trailers written when hashed (no parking): the reference
              // image of the parked-trailer product seal (tests/test_sst4k.py)
      if (!seal) return hipErrorInvalidValue;
      hipLaunchKernelGGL((crc_sst4k_kernel<SstSrc, SealSink, true>), grid, block, 0, s, d_tables, src, n, SealSink{});
      return hipGetLastError();
    case 18:  // the hooks on the 32-B-piece any-length stream kernel: an independent kernel for the
              // reference-file tests (tests/test_sst_files.py)
      if (seal)
        hipLaunchKernelGGL((crc_stream_kernel<SstSrc, SealSink, 0, true, true>), grid, block, 0, s, d_tables, src, n,
                           SealSink{});
      else
        hipLaunchKernelGGL((crc_stream_kernel<SstSrc, SstVerifySink, 0, true, true>), grid, block, 0, s, d_tables,
                           src, n, SstVerifySink{ok, nbad});
      return hipGetLastError();
    default:  // 0: the product routing
      return launch_sst(g, d_tables, buf, buf_len, h, n, seal, ok, nbad, s);
  }
}

hipError_t launch_fixed_variant(int v, const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                                uint64_t stride, uint32_t len, uint64_t nblk, uint32_t flags, uint32_t init,
                                uint32_t* out, hipStream_t s) {
  if (v == 16) {  // the any-length kernel for every length and alignment (16-B pieces, nt, packed trees)
    const dim3 grid(grid_for(g, nblk)), block(kThreads);
    const FixedSrc src{base, stride, len, (flags & PDB_CRC_USE_INIT) ? ~init : 0xFFFFFFFFu};
    const bool aligned4 = ((reinterpret_cast<uintptr_t>(base) + (len & 15u)) & 3u) == 0 && (stride & 3u) == 0;
    if (aligned4)
      hipLaunchKernelGGL((crc_stream16_kernel<FixedSrc, OutSink, true, true, true>), grid, block, 0, s, d_tables, src,
                         nblk, OutSink{out, flags});
    else
      hipLaunchKernelGGL((crc_stream_kernel<FixedSrc, OutSink, 0, true, true>), grid, block, 0, s, d_tables, src, nblk,
                         OutSink{out, flags});
    return hipGetLastError();
  }
  return launch_fixed(g, d_tables, base, stride, len, nblk, flags, init, out, s);  // 0: the product routing
}

hipError_t launch_desc_variant(int v, const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                               const pdb_blk* blk, uint64_t nblk, uint32_t flags, uint32_t* out, hipStream_t s) {
  if (nblk == 0) return hipSuccess;
  const dim3 grid(grid_for(g, nblk)), block(kThreads);
  const DescSrc src{base, blk, flags};
  const OutSink sink{out, flags};
  const bool mixed = (flags & PDB_CRC_SIZE_MIXED) != 0;
  switch (v) {
    case 16:  // size hints ignored: the any-length kernel (the product's C3 routing) for every list
      hipLaunchKernelGGL((crc_stream16_kernel<DescSrc, OutSink, true, true, true, QuadTabs, true>), grid, block, 0, s,
                         d_tables, src, nblk, sink);
      return hipGetLastError();
    case 161:  // the C3 routing's loads, scheduling and byte-balanced ranges with NO hash (its pattern
               // ceiling, bench.py pattern_ceiling; wrong CRCs by design)
      hipLaunchKernelGGL((crc_stream16_kernel<DescSrc, OutSink, true, true, true, QuadTabs, true, true, true>), grid, block,
                         0, s, d_tables, src, nblk, sink);
      return hipGetLastError();
    // the record kernel (size-hinted lists): its parts, its cross-checks and its work distribution
    case 63:  // loads and staging alone (no hash; results undefined)
      return launch_lanespan<DescSrc, OutSink, 1>(g, d_tables, src, nblk, record_class(flags), sink, s, mixed);
    case 64:  // the hash alone over stale staging (no loads; results undefined)
      return launch_lanespan<DescSrc, OutSink, 2>(g, d_tables, src, nblk, record_class(flags), sink, s, mixed);
    case 67:  // the bookkeeping alone (no loads, no hash)
      return launch_lanespan<DescSrc, OutSink, 3>(g, d_tables, src, nblk, record_class(flags), sink, s, mixed);
    case 127:  // pricing: the hash's fold operators as plain XORs (no lookups)
      return launch_lanespan<DescSrc, OutSink, 43>(g, d_tables, src, nblk, record_class(flags), sink, s, mixed);
    case 128:  // pricing: each fold operator as 8 conflict-free table lookups
      return launch_lanespan<DescSrc, OutSink, 44>(g, d_tables, src, nblk, record_class(flags), sink, s, mixed);
    case 129:  // pricing: the fold operators' lookups with no dependence between them
      return launch_lanespan<DescSrc, OutSink, 45>(g, d_tables, src, nblk, record_class(flags), sink, s, mixed);
    case 130:  // pricing: the cross-lane fold operators as plain XORs
      return launch_lanespan<DescSrc, OutSink, 46>(g, d_tables, src, nblk, record_class(flags), sink, s, mixed);
    case 131:  // pricing: the staging stores as one 16-B store per lane and item
      return launch_lanespan<DescSrc, OutSink, 47>(g, d_tables, src, nblk, record_class(flags), sink, s, mixed);
    case 132:  // pricing: the chains' words as 16-B LDS reads
      return launch_lanespan<DescSrc, OutSink, 48>(g, d_tables, src, nblk, record_class(flags), sink, s, mixed);
    case 133:  // exact: the cross-lane pre-shift's lookups on the lanes that use them only (EXEC-masked)
      return launch_lanespan<DescSrc, OutSink, 49>(g, d_tables, src, nblk, record_class(flags), sink, s, mixed);
    case 134:  // exact: each part hashed as four chains (three in-part folds: the round-5 form, MODE 52)
      return launch_lanespan<DescSrc, OutSink, 52>(g, d_tables, src, nblk, record_class(flags), sink, s, mixed);
    case 125:  // exact: the batch-uniform k only (no per-record lanes for mixed sizes)
      return launch_lanespan<DescSrc, OutSink, 17>(g, d_tables, src, nblk, record_class(flags), sink, s, mixed);
    case 126:  // the item geometry per record instead of its CRC (MODE 18; tests/test_lanespan.py)
      return launch_lanespan<DescSrc, OutSink, 18>(g, d_tables, src, nblk, record_class(flags), OutSink{out, 0u}, s,
                                                   mixed);
    case 180:    // the product / loads + staging alone / hash alone, + per-wave [start, end] s_memrealtime
    case 181:    // and [start, end] s_memtime stamps at out + nblk rounded up to 8 B (the caller sizes
    case 182: {  // `out` for 4 x 8 B per wave; tools/span_clock.py)
      StampOutSink ss;
      ss.out = out;
      ss.flags = flags;
      ss.stamps = reinterpret_cast<uint64_t*>(out + ((nblk + 1u) & ~1ull));
      if (v == 180) return launch_lanespan<DescSrc, StampOutSink, 40>(g, d_tables, src, nblk, record_class(flags), ss, s, mixed);
      if (v == 181) return launch_lanespan<DescSrc, StampOutSink, 41>(g, d_tables, src, nblk, record_class(flags), ss, s, mixed);
      return launch_lanespan<DescSrc, StampOutSink, 42>(g, d_tables, src, nblk, record_class(flags), ss, s, mixed);
    }
    default:  // 0 (and unknown ids): the shipped routing
      return launch_desc(g, d_tables, base, blk, nblk, flags, kModeOut, nullptr, out, nullptr, nullptr, s);
  }
}

hipError_t launch_read_stream(const uint8_t* base, uint64_t nbytes, uint32_t* out, hipStream_t s) {
  const uint64_t n16 = nbytes / 16;
  hipLaunchKernelGGL(read_stream_kernel, dim3(256 * 16), dim3(256), 0, s,
                     reinterpret_cast<const u32x4*>(base), n16, out);
  return hipGetLastError();
}

hipError_t launch_read_pattern4k(const LaunchGeom& g, const uint8_t* base, uint64_t nblk,
                                 int variant, uint32_t* out, hipStream_t s) {
  if (variant != 21) return hipErrorInvalidValue;  // the 4-KiB path's pattern (the others: round 1-2, removed)
  hipLaunchKernelGGL(read_pattern4k_kernel, dim3(g.grid), dim3(kThreads), 0, s, base, nblk, out);
  return hipGetLastError();
}

hipError_t launch_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset, hipStream_t s) {
  if (nbytes == 0) return hipSuccess;
  uint64_t blocks = ((nbytes + 7) / 8 + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(fill_splitmix_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, dst, nbytes, seed,
                     byte_offset);
  return hipGetLastError();
}

}  // namespace pdb
