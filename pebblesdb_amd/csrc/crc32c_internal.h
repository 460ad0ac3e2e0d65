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

// ---- the long-block lane (device-resident batches) ----------------------------------------------
// A batch kernel hashes each block on one wave (~2 GB/s), so one index or filter block of a few MiB
// inside a batch of 4-KiB blocks would set the launch's length (a 4 MiB block: ~2 ms against ~3 us
// for 16 MiB of data blocks).  Instead the wave that meets a block of >= its kernel's threshold
// EXPORTS it: one atomic reserves a record and the block's pieces in a per-stream scratch, and the
// wave writes the piece list -- a head of h = n - 4096 m bytes (1..4096, Value() seed) followed by m
// pieces of exactly 4096 B (hashed from state 0) -- and goes on.  After the batch kernel, on the same
// stream, crc_longpiece_kernel hashes every exported piece on the whole GPU (the sstable-sized
// kernel's 4-KiB body path: ~HBM rate), and long_combine_kernel folds each record's leaves with the
// power-of-two operators (R(H || S_1 .. S_m) = sum_j shift(leaf_j, 4096 (m - j)), zero leaves padded
// in front) and hands the raw state to the batch's own sink, exactly where the batch kernel would
// have.  A full scratch (or no scratch) leaves the block to the batch kernel's one-wave path: the
// results never depend on the lane, only the time does.  The combine kernel's last workgroup resets
// the counters, so the lane is allocation-free and capturable per call.
struct LongRec {     // 32 B
  uint64_t i;        // block index in the batch
  uint64_t p;        // block address
  uint32_t n;        // bytes under the CRC
  uint32_t init_raw; // ~Extend seed (0xFFFFFFFF: Value)
  uint32_t q0, np;   // its pieces (= leaves) q0 .. q0 + np - 1, the head first
};
struct LongPiece {   // 16 B
  uint64_t p;
  uint32_t n;        // 4096, or the head's 1..4096
  uint32_t seeded;   // 1: the head (Value() seed), 0: a full piece (state 0)
};
struct LongLane {
  unsigned long long* hdr;  // [0] = records << 40 | pieces reserved; [1] = combine workgroups done
  LongRec* rec;
  LongPiece* piece;
  uint32_t* leaf;           // raw state of piece q
  const uint32_t* pow2;     // the 64 power-of-two shift operators (1024 u32 each)
  uint32_t rec_cap, piece_cap;
};
constexpr uint32_t kLongRecCap = 1u << 16;
constexpr uint32_t kLongPieceCap = 1u << 21;  // 8 GiB of long blocks per call
constexpr unsigned long long kLongPieceMask = (1ull << 40) - 1;
constexpr uint32_t kLongMinBytes = 16u << 10;         // sstable-sized and record kernels
constexpr uint32_t kLongMinStream = (64u << 10) + 1;  // the any-length stream kernel (C3's 1..64 KiB stay)
// scratch layout: [hdr 256 B][records][pieces][leaves] (a batch kernel carries only the base)
constexpr size_t kLongHdrBytes = 256;
constexpr size_t kLongRecOff = kLongHdrBytes;
constexpr size_t kLongPieceOff = kLongRecOff + size_t(kLongRecCap) * sizeof(LongRec);
constexpr size_t kLongLeafOff = kLongPieceOff + size_t(kLongPieceCap) * sizeof(LongPiece);
constexpr size_t long_scratch_bytes() { return kLongLeafOff + size_t(kLongPieceCap) * 4; }
// The lane over a zeroed scratch of long_scratch_bytes() at d (null d: no lane).
LongLane long_lane_at(uint8_t* d, const uint32_t* d_pow2);

// crc32c_kernels.hip -- all launches are asynchronous on `s`.  `ll`: the long-block lane (null: none;
// every block is then hashed by the batch kernel itself).
hipError_t launch_fixed(const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                        uint64_t stride, uint32_t len, uint64_t nblk, uint32_t flags, uint32_t init,
                        uint32_t* out, hipStream_t s);
hipError_t launch_desc(const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                       const pdb_blk* blk, uint64_t nblk, uint32_t flags, int mode,
                       const uint32_t* expected, uint32_t* out, uint8_t* ok, uint32_t* nbad,
                       hipStream_t s, const LongLane* ll = nullptr);
hipError_t launch_sst(const LaunchGeom& g, const uint32_t* d_tables, uint8_t* buf, uint64_t buf_len,
                      const pdb_block_handle* h, uint64_t n, bool seal, uint8_t* ok, uint32_t* nbad,
                      hipStream_t s, const LongLane* ll = nullptr);
// out[i] = Mask(crc32c(contents_i || type_i)) -- the trailer word a seal writes, as an array.
hipError_t launch_sst_masked(const LaunchGeom& g, const uint32_t* d_tables, uint8_t* buf, uint64_t buf_len,
                             const pdb_block_handle* h, uint64_t n, uint32_t* out, hipStream_t s,
                             const LongLane* ll = nullptr);
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
