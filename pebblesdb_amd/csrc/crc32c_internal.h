// crc32c_internal.h -- declarations shared between the C-ABI layer and the HIP kernel TU.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "../../include/pdb_crc32c.h"

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
// span_scratch_words(n) u32.  *out = Extend(init, data[0..n)).
uint64_t span_scratch_words(uint64_t n);
hipError_t launch_span(const LaunchGeom& g, const uint32_t* d_tables, const uint32_t* d_pow2,
                       uint32_t init, const uint8_t* data, uint64_t n, uint32_t* scratch, uint32_t* out,
                       hipStream_t s);

// crc32c_server.hip -- the scalar Extend service (persistent one-workgroup kernel).  Two boxes:
// the request box `in` (request word + the caller's bytes, placed so that they end on a 16-B
// boundary: data = in + sizeof(ServerBox) + ((-n) & 15)) lives in fine-grained device memory the
// host writes through the large BAR (the GPU then polls and reads local HBM), or in pinned host
// memory when the BAR is small; the response box `out` (resp word, exit_epoch) is pinned host
// memory the GPU writes across PCIe.
//   req  (host -> device, one 64-bit word, so one poll reads a whole request):
//        bits 0..31 init (the Extend seed), 32..48 len (<= kServerCap, or kServerStop),
//        49..63 seq (15 bits, bumped per request)
//   resp (device -> host, one 64-bit word): bits 0..31 crc, 32..46 seq of the answered request
//   exit_epoch: epoch of the last server instance that has left its loop
struct ServerBox {
  uint64_t req;
  uint64_t pad0[7];
  uint64_t resp;
  uint32_t exit_epoch;
  uint32_t pad1[13];
  // written at exit (diagnostics): requests served, ticks (10 ns) from seeing a request to
  // issuing its answer, polls, lifetime ticks
  uint64_t stat_requests, stat_serve_ticks, stat_polls, stat_life_ticks;
  uint64_t pad2[12];
};
static_assert(sizeof(ServerBox) == 256, "mailbox is 4 cache lines");
constexpr uint32_t kServerCap = 64u << 10;  // largest request the server takes
constexpr uint32_t kServerStop = 0x1FFFFu;  // len value of a stop request
constexpr uint32_t kServerSeqMask = 0x7FFFu;
constexpr size_t kServerBytes = sizeof(ServerBox) + kServerCap + 16;
// served0: the seq the new instance treats as already answered.
hipError_t launch_server(const uint32_t* d_tables, ServerBox* d_in, ServerBox* d_out, uint32_t epoch,
                         uint32_t served0, uint64_t idle_ticks, uint64_t life_ticks, hipStream_t s);

}  // namespace pdb
