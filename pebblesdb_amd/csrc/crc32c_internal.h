// crc32c_internal.h -- declarations shared between the C-ABI layer and the HIP kernel TU.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "../../include/pdb_crc32c.h"
#include "crc32c_math.h"

namespace pdb {

// crc32c_tables.cpp
void build_byte_table(uint32_t t0[256]);
void build_device_tables(uint32_t* out);  // PDB_TABLE_WORDS
void build_pow2_tables(uint32_t* out);    // PDB_POW2_WORDS
uint32_t host_shift(uint32_t c, uint64_t nbytes);

// Kernel launch modes for the descriptor kernel.
enum DescMode : int {
  kModeOut = 0,     // out[i] = crc
  kModeVerify = 1,  // ok[i] = (crc == expected[i])
};

struct LaunchGeom {
  uint32_t grid;   // workgroups (one per CU: the LDS image is ~156 KiB)
  uint32_t block;  // threads per workgroup
};

// crc32c_kernels.hip -- all launches are asynchronous on `s`.
hipError_t launch_fixed(const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                        uint64_t stride, uint32_t len, uint64_t nblk, uint32_t flags, uint32_t init,
                        uint32_t* out, hipStream_t s);
hipError_t launch_desc(const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                       const pdb_blk* blk, uint64_t nblk, uint32_t flags, int mode,
                       const uint32_t* expected, uint32_t* out, uint8_t* ok, uint32_t* nbad,
                       hipStream_t s);
hipError_t launch_sst(const LaunchGeom& g, const uint32_t* d_tables, uint8_t* buf, uint64_t buf_len,
                      const pdb_block_handle* h, uint64_t n, bool seal, uint8_t* ok, uint32_t* nbad,
                      hipStream_t s);
// out[i] = Mask(crc32c(contents_i || type_i)) -- the trailer word a seal writes, as an array.
hipError_t launch_sst_masked(const LaunchGeom& g, const uint32_t* d_tables, uint8_t* buf, uint64_t buf_len,
                             const pdb_block_handle* h, uint64_t n, uint32_t* out, hipStream_t s);
// Long span: raw CRCs of `nseg` segments of 2^seg_log2 bytes (+ the tail) in parallel, then a
// one-workgroup tree combine with the power-of-two operators.  `scratch` holds
// span_scratch_words(n) u32.  *out = Extend(init, data[0..n)).  Segments of at least
// 2^min_seg_log2 bytes (4 KiB for a block read across PCIe: one round trip per wave).
uint64_t span_scratch_words(uint64_t n, uint32_t min_seg_log2 = PDB_SPAN_MIN_SEG_LOG2);
hipError_t launch_span(const LaunchGeom& g, const uint32_t* d_tables, const uint32_t* d_pow2,
                       uint32_t init, const uint8_t* data, uint64_t n, uint32_t* scratch, uint32_t* out,
                       hipStream_t s, uint32_t min_seg_log2 = PDB_SPAN_MIN_SEG_LOG2);
// Many spans in two launches: `pieces` (npieces descriptors over `base`, PDB_CRC_USE_INIT) are
// every span's leaves in order -- its first piece with init 0 (the Value seed), then pieces of
// exactly 2^seg_log2 bytes with init 0xFFFFFFFF (raw state 0) -- and parts[b] = {span b's first
// leaf, its leaves (<= 2^PDB_SPAN_MAX_SEGS_LOG2), ceil(log2(leaves))}; out[b] = Value(span b).
// `leaves` holds npieces u32.
struct SpanPart {
  uint32_t leaf0, nleaves, m_log2, pad;
};
hipError_t launch_span_many(const LaunchGeom& g, const uint32_t* d_tables, const uint32_t* d_pow2, const uint8_t* base,
                            const pdb_blk* pieces, uint64_t npieces, const SpanPart* parts, uint32_t nparts,
                            uint32_t seg_log2, uint32_t* leaves, uint32_t* out, hipStream_t s);

// crc32c_server.hip -- the scalar Extend service: ONE persistent workgroup of kServerWaves waves
// serving kServerSlots request slots, so concurrent callers (the engine's writer, memtable,
// compaction and reader threads: db/db_impl.cc:235-239) each post into their own slot without a
// global lock, and up to kServerWaves requests are hashed at once.
//   request area `in` (host -> device; fine-grained device memory the host writes through the
//   large BAR, else pinned host memory):
//     [0, 256)           ServerCtl: `stop`, bumped by the host to make the instance leave
//     [256, 768)         req word of slot s at 256 + 8 s: bits 0..31 init (the Extend seed),
//                        32..48 len (<= kServerCap), 49..63 seq (15 bits, bumped per request)
//     [1024, ...)        slot s's bytes in kSlotStride-byte areas, placed so that they END on a
//                        16-B boundary: data = in + kSlotDataOff + s kSlotStride + ((-n) & 15)
//   response area `out` (device -> host, pinned host memory):
//     resp word of slot s at 64 s (own cache line): bits 0..31 crc, 32..46 seq answered
//     ServerExit at kExitOff: the epoch of the last instance that has left, and its counters
// A request is pending while its slot's req seq differs from the resp seq, so an instance starts
// by reading the resp words: requests an earlier instance left behind are served at once.
constexpr uint32_t kServerSlots = 64;
constexpr uint32_t kServerWaves = 16;        // wave w polls slots w, w + 16, w + 32, w + 48
constexpr uint32_t kServerCap = 64u << 10;   // largest request the service takes
constexpr uint32_t kServerSeqMask = 0x7FFFu;
constexpr size_t kSlotStride = kServerCap + 256;
constexpr size_t kReqOff = 256;
constexpr size_t kSlotDataOff = 1024;
constexpr size_t kServerInBytes = kSlotDataOff + kServerSlots * kSlotStride;
struct ServerCtl {
  uint64_t stop;
  uint64_t pad[31];
};
struct ServerExit {
  uint32_t exit_epoch;
  uint32_t pad0;
  // diagnostics, written at exit: requests served, ticks (10 ns) from seeing a request to issuing
  // its answer, polls (all waves), lifetime ticks
  uint64_t stat_requests, stat_serve_ticks, stat_polls, stat_life_ticks;
  uint64_t pad1[27];
};
static_assert(sizeof(ServerCtl) == 256 && sizeof(ServerExit) == 256, "mailbox records are 4 cache lines");
constexpr size_t kExitOff = kServerSlots * 64;
constexpr size_t kServerOutBytes = kExitOff + sizeof(ServerExit);
// stop0: the ctl->stop value this instance runs under (it leaves when the word changes)
// stamps != 0 (diagnostics, PDB_SERVER_STAMPS): each answer's response line also carries the poll
// and hash-done ticks (s_memrealtime) in its words 1 and 2.
hipError_t launch_server(const uint32_t* d_tables, uint8_t* d_in, uint8_t* d_out, uint32_t epoch, uint64_t stop0,
                         uint64_t idle_ticks, uint64_t life_ticks, uint32_t stamps, hipStream_t s);

}  // namespace pdb
