// integration/pdb_hooks.h -- counters of the engine-side hooks (pdb_table_builder.cc: batched
// WriteRawBlock seals; pdb_format.cc: ReadBlock verifies), read by the db_bench-equivalent harness
// (pdb_dbbench.cc) to report the GPU CRC's share of a run and its copy-inclusive rate.
#ifndef PDB_INTEGRATION_HOOKS_H_
#define PDB_INTEGRATION_HOOKS_H_

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
  uint64_t verify_failed;  // Corruption("block checksum mismatch") returned
} pdb_hook_stats;

void pdb_hook_stats_get(pdb_hook_stats* out);
void pdb_hook_stats_reset(void);

#ifdef __cplusplus
}

namespace pdb_hooks {
// internal: the hooks add to the counters (thread-safe, relaxed atomics)
void AddSeal(uint64_t blocks, uint64_t bytes, uint64_t ns);
void AddVerify(uint64_t bytes, uint64_t ns, bool failed);
uint64_t NowNs();
}  // namespace pdb_hooks
#endif

#endif  // PDB_INTEGRATION_HOOKS_H_
