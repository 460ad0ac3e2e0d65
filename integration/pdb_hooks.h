// integration/pdb_hooks.h -- counters of the engine-side hooks (pdb_table_builder.cc: batched
// WriteRawBlock seals; pdb_format.cc: ReadBlock verifies; pdb_table.cc: scan read-ahead batches),
// read by the db_bench-equivalent harness (pdb_dbbench.cc) to report the GPU CRC's share of a run
// and its copy-inclusive rate; and ReadBlock's block decoding, shared with pdb_table.cc.
#ifndef PDB_INTEGRATION_HOOKS_H_
#define PDB_INTEGRATION_HOOKS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pdb_hook_stats {
  uint64_t seal_calls;     // pdb_sst_seal_host batches issued by TableBuilders
  uint64_t seal_blocks;    // blocks (trailers) sealed
  uint64_t seal_bytes;     // block bytes + trailers shipped to the GPU
  uint64_t seal_ns;        // wall time inside the seal calls (H2D + kernel + D2H + trailer encode)
  uint64_t verify_calls;   // ReadBlock checksum checks on the GPU
  uint64_t verify_bytes;   // contents + type bytes checked
  uint64_t verify_ns;      // wall time inside them
  uint64_t verify_failed;  // Corruption("block checksum mismatch") returned (or found by a scan batch)
  uint64_t scan_batches;   // pdb_table.cc: verified read-ahead batches (pdb_sst_verify_host) of scans
  uint64_t scan_blocks;    // data blocks checked in them
  uint64_t scan_bytes;     // bytes read and checked
  uint64_t scan_ns;        // wall time of the window reads + GPU checks
  uint64_t seal_busy_ns;   // wall time with at least one seal call in flight (builders seal concurrently)
  uint64_t seal_overlap;   // most seal calls in flight at once
  // the seal calls by batch size (< 1, 1-4, 4-8, 8-15, >= 15 MiB): calls, bytes, call time (ns)
  uint64_t seal_size_calls[5];
  uint64_t seal_size_bytes[5];
  uint64_t seal_size_ns[5];
} pdb_hook_stats;

void pdb_hook_stats_get(pdb_hook_stats* out);
void pdb_hook_stats_reset(void);

#ifdef __cplusplus
}

namespace pdb_hooks {
// internal: the hooks add to the counters (thread-safe, relaxed atomics)
void AddSeal(uint64_t blocks, uint64_t bytes, uint64_t ns);
// around every seal call: the union of the calls' intervals (seal_busy_ns) and their overlap
void SealBegin();
void SealEnd();
void AddVerify(uint64_t bytes, uint64_t ns, bool failed);
void AddScan(uint64_t blocks, uint64_t bytes, uint64_t ns, uint64_t bad);
uint64_t NowNs();
}  // namespace pdb_hooks

namespace leveldb {
struct BlockContents;
class Status;
}  // namespace leveldb
namespace pdb_hooks {
leveldb::Status BlockFromChecked(const char* data, size_t n, char* owned, bool stable, leveldb::BlockContents* result);
}  // namespace pdb_hooks
#endif

#endif  // PDB_INTEGRATION_HOOKS_H_
