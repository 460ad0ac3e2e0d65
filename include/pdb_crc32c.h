/*
 * pdb_crc32c.h -- C-ABI drop-in boundary for PebblesDB's sstable block checksum path,
 * served by hand-written HIP kernels for MI355X (gfx950).
 *
 * Reference interfaces this replaces (paths under utsaslab/pebblesdb src/):
 *   util/crc32c.h:17      uint32_t crc32c::Extend(uint32_t init_crc, const char* data, size_t n)
 *   util/crc32c.h:20-22   uint32_t crc32c::Value(const char* data, size_t n)
 *   util/crc32c.h:29-32   uint32_t crc32c::Mask(uint32_t crc)    (ror32(crc,15) + 0xa282ead8)
 *   util/crc32c.h:35-40   uint32_t crc32c::Unmask(uint32_t masked)
 *   util/crc32c.cc:65,99  the file-static crc32c_func pointer = the reference's only swap point
 *   table/table_builder.cc:187-205  TableBuilder::WriteRawBlock: trailer [type][Mask(crc(contents||type))]
 *   table/format.cc:66-104          ReadBlock: Unmask(DecodeFixed32(data+n+1)) == Value(data, n+1)
 *                                   else Status::Corruption("block checksum mismatch")
 *   table/format.h:87               kBlockTrailerSize = 5
 *
 * Conventions
 *   - Plain C types only; device pointers are `const void*`, streams are `void*` (a hipStream_t;
 *     NULL = the HIP default stream, as for hipLaunchKernel).  Host entry points use a
 *     per-device internal stream and return after the results are in host memory.
 *   - Every batch entry returns 0 or a negative PDB_E* code.  There is NO CPU fallback: with no
 *     usable device the call fails (PDB_ENODEV) and pdb_last_error() says why.
 *   - Scalar Extend/Value cannot report errors (the reference contract, util/crc32c.h:17); on a
 *     device failure they abort() with a message instead of returning a wrong value.
 *   - Caller owns every buffer.  Device-resident entry points are stream-ordered and capturable
 *     into a hipGraph; the only memory they own is the long-block lane's scratch (~42 MiB per
 *     caller stream, made at the stream's first call outside a capture or by
 *     pdb_crc32c_prepare_stream, kept for the process).  Host entry points stage through a cached
 *     per-device workspace that only grows.
 *   - Long blocks (the long-block lane): a block of >= 16 KiB in an sstable batch or a
 *     PDB_CRC_SIZE_4K descriptor batch (> 64 KiB in a descriptor batch without a size hint) is not
 *     hashed by the wave that meets it; it is split into 4-KiB pieces hashed on the whole GPU after
 *     the batch kernel and folded with shift operators, on the same stream.  (Descriptor batches
 *     with a WAL-record hint -- _256 / _512 / _1023 / _1K -- take no lane: log records are <= 32 KiB.)  Results are identical either way: a stream without a
 *     lane (captured before it was prepared), or a call whose long blocks exceed the scratch (8 GiB
 *     of them, or 65536 blocks), hashes them on one wave each -- only the time differs.
 *   - Per-block length in batches is < 2^32 bytes (the reference narrows to uint32_t:
 *     util/crc32c.cc:19-23,589); a single span (pdb_crc32c_extend*) may be longer.
 *   - Thread-safe: host entry points take one of 4 staging contexts per device; device entry points
 *     are pure launches.
 *   - Every result depends only on the arguments.  The ROUTE (never the result) also depends on
 *     pdb_crc32c_init_mask (which devices host batches stage through) and on these environment
 *     variables, each read once per process, for experiments and diagnostics:
 *       PDB_HOST_CHUNK_BYTES  host staging group span (default 256 MiB)
 *       PDB_HOST_MAPPED=0     sstable host batches in pdb_host_alloc memory take the DMA route,
 *                             not zero-copy
 *       PDB_LONG_BLOCK=<n>    host sstable batches: the split threshold of long blocks (16 KiB)
 *       PDB_SCALAR_WAIT=poll|sync  scalar Extend launches per call instead of the persistent server
 *       PDB_SERVER_BOX=host   the scalar server's request area in pinned host memory, not in
 *                             device memory through the large BAR
 *       PDB_SEAL_STAMPS=<path>, PDB_SERVER_STAMPS=<path>  per-call timestamps written at exit
 *   - Device-resident batches may read a few bytes outside a block: up to 15 bytes before its first
 *     byte and up to 3 bytes past its last one, never outside the 4-B-aligned dwords and 16-B lines
 *     that hold the block's bytes.  A buffer handed to a device entry point must therefore stay
 *     readable to the 16-B boundaries around every block (any hipMalloc'd or torch allocation
 *     does); the bytes outside a block never affect its CRC.  Descriptor batches with the
 *     PDB_CRC_SIZE_256 / _512 / _1023 / _1K hints (and fixed strides of 1..1152 B) also read the gaps of
 *     at most 64 bytes between consecutive blocks of the list (a log image's record headers and
 *     block trailers), and only those: a larger gap, or a block out of ascending order, starts a
 *     new load run.
 *   - Host batches stage at most 256 MiB of span per device copy (PDB_HOST_CHUNK_BYTES, read once
 *     per process, overrides it); the copies of one group overlap the kernel of the previous one.
 *   - Bench / test infrastructure (synthetic input, A/B kernel variants, roofline calibration)
 *     lives in a separate library, include/pdb_crc32c_diag.h; nothing here depends on it.
 */
#ifndef PDB_CRC32C_H_
#define PDB_CRC32C_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: pdb_crc32c_prepare_stream, pdb_crc32c_init_mask and pdb_host_stripe_plan added;
 *    pdb_sst_seal_device_scratch (version 1) removed */
#define PDB_CRC32C_ABI_VERSION 2

/* One block of a batch: bytes [base+off, base+off+len), optional Extend seed. 16 bytes. */
typedef struct pdb_blk {
  uint64_t off;  /* byte offset from the batch base (any alignment) */
  uint32_t len;  /* bytes under the CRC */
  uint32_t init; /* Extend() init crc; used only with PDB_CRC_USE_INIT */
} pdb_blk;

/* An sstable BlockHandle (table/format.h:22-45): block contents at [offset, offset+size),
 * followed by the 5-byte trailer [type][masked crc LE32] at offset+size. */
typedef struct pdb_block_handle {
  uint64_t offset;
  uint64_t size;
} pdb_block_handle;

/* flags */
#define PDB_CRC_MASK_OUTPUT 0x1u /* out[i] = Mask(crc) (util/crc32c.h:29-32) */
#define PDB_CRC_USE_INIT 0x2u    /* crc = Extend(blk.init, ...) instead of Value(...) */
/* Size-class hints for descriptor batches (speed only: results are identical with or without;
 * ignored with PDB_CRC_USE_INIT).  Host batch entries pick the class themselves from the lengths. */
#define PDB_CRC_SIZE_1K 0x4u /* most blocks 1024..1152 B: WAL physical records (type || fragment) */
#define PDB_CRC_SIZE_4K 0x8u /* most blocks 4096..4352 B: sstable data blocks (contents || type) */
#define PDB_CRC_SIZE_256 0x10u /* most blocks 1..256 B: small WAL / MANIFEST records */
#define PDB_CRC_SIZE_512 0x20u /* most blocks 257..512 B: WAL records of ~400-B values */
#define PDB_CRC_SIZE_1023 0x40u /* most blocks 513..1023 B: WAL records of ~500..990-B values */
/* With PDB_CRC_SIZE_512 / _1023: the lengths vary within the class (records of varied values), so
 * each record is hashed on as many lanes as its own length needs instead of the batch's longest
 * record's (+10..50 % on such logs; about -2 % on logs of equal records, so it is a hint).  Host
 * batch entries set it themselves from the lengths. */
#define PDB_CRC_SIZE_MIXED 0x80u

/* error codes */
#define PDB_OK 0
#define PDB_ENODEV (-1)  /* no HIP device / extension unusable */
#define PDB_EHIP (-2)    /* HIP runtime error (see pdb_last_error) */
#define PDB_EINVAL (-3)  /* bad argument */
#define PDB_ERANGE (-4)  /* a block or buffer exceeds a limit */
#define PDB_ENOMEM (-5)  /* device workspace allocation failed */

/* ---- library / device ---------------------------------------------------------------------- */
int pdb_crc32c_abi_version(void);
/* Create the per-device state: upload the CRC tables, query CU count, create the internal
 * stream.  Called implicitly by every entry point; explicit calls are idempotent. */
int pdb_crc32c_init(int device);
const char* pdb_last_error(void); /* thread-local message of the last failure */
/* The devices host batches stripe over (SURVEY §8(b) init(device_mask); bit d = HIP device d):
 * pdb_crc32c_batch_host / _verify_host and the staging (DMA) route of pdb_sst_seal_host /
 * _verify_host split a batch into contiguous runs of staging groups, ~1/N of the bytes per device,
 * and stage every run through its own device's PCIe link at once (a batch of less than 8 MiB per
 * device uses fewer devices).  Device-resident entry points and the zero-copy route keep the
 * calling thread's device.  0 (the default) = the calling thread's current device.  Makes every
 * masked device's state now; returns the number of devices, or a negative error (PDB_EINVAL: a
 * device that is not visible). */
int pdb_crc32c_init_mask(uint64_t device_mask);
/* The staging plan a host descriptor batch of these blocks gets over `ndev` devices (groups of at
 * most `chunk_bytes` of span, 0 = the library's 256 MiB): group k starts at block group_first[k] and
 * runs on device index group_dev[k].  Fills at most `cap` groups; returns the number of groups.  Pure
 * host code (no device needed): the planning half of pdb_crc32c_init_mask's striping, for tests. */
int64_t pdb_host_stripe_plan(const pdb_blk* blk, uint64_t nblk, uint32_t ndev, uint64_t chunk_bytes,
                             uint64_t* group_first, uint32_t* group_dev, uint64_t cap);
/* Make the long-block lane's scratch for device-resident calls on `stream` now (it is otherwise made
 * at the stream's first call): call it before capturing device entry points on a stream into a
 * hipGraph.  PDB_EINVAL while the stream is capturing. */
int pdb_crc32c_prepare_stream(void* stream);
/* Device the calling thread uses (HIP current device). */
int pdb_crc32c_current_device(void);

/* ---- scalar, LevelDB-compatible (util/crc32c.h:17-40) ---------------------------------------- */
uint32_t pdb_crc32c_extend(uint32_t init_crc, const void* data, size_t n); /* host data; spans
                                                                             >= 8 MiB are split */
uint32_t pdb_crc32c_value(const void* data, size_t n);                     /* host data */
uint32_t pdb_crc32c_mask(uint32_t crc);
uint32_t pdb_crc32c_unmask(uint32_t masked_crc);

/* ---- long spans ------------------------------------------------------------------------------
 * One span of any length (up to 2^45 bytes, so also past the reference's silent 4 GiB length
 * narrowing, util/crc32c.cc:19-23): hashed as up to 16384 segments in parallel, folded on the
 * device.  *d_out = Extend(init_crc, d_data[0..n)).  d_scratch: >= extend_scratch_words(n) u32. */
uint64_t pdb_crc32c_extend_scratch_words(uint64_t n);
int pdb_crc32c_extend_device(uint32_t init_crc, const void* d_data, uint64_t n, uint32_t* d_scratch,
                             uint64_t scratch_words, uint32_t* d_out, void* stream);

/* ---- device-resident batches (the hot path) ------------------------------------------------ */
/* Blocks i in [0,nblk): bytes [d_base + i*stride, +len).  Seed `init` applies to every block when
 * PDB_CRC_USE_INIT is set.  d_out[i] = crc (masked with PDB_CRC_MASK_OUTPUT). */
int pdb_crc32c_batch_device_fixed(const void* d_base, uint64_t stride, uint32_t len, uint64_t nblk,
                                  uint32_t flags, uint32_t init, uint32_t* d_out, void* stream);
/* Blocks from a device-resident descriptor array. */
int pdb_crc32c_batch_device(const void* d_base, const pdb_blk* d_blk, uint64_t nblk, uint32_t flags,
                            uint32_t* d_out, void* stream);
/* Verify: d_ok[i] = (crc_i == expected_i), where expected is masked iff PDB_CRC_MASK_OUTPUT.
 * *d_nbad (device u32, caller-zeroed) is atomically incremented per mismatch; may be NULL. */
int pdb_crc32c_verify_device(const void* d_base, const pdb_blk* d_blk, uint64_t nblk, uint32_t flags,
                             const uint32_t* d_expected, uint8_t* d_ok, uint32_t* d_nbad,
                             void* stream);

/* ---- pinned host staging -----------------------------------------------------------------------
 * Page-locked, device-mapped host memory for a caller that stages the blocks of host batches
 * (integration/pdb_table_builder.cc stages its sealed batches in it).  pdb_sst_seal_host /
 * pdb_sst_verify_host on a buffer inside one such allocation run zero-copy: the kernel reads the
 * blocks (and a seal writes the trailers) through the mapping, one launch, no DMA; the other host
 * entry points DMA from it without the runtime's pageable bounce copies.  Any host memory stays
 * valid for every entry point; this only changes the rate.  Freed allocations are kept for reuse
 * (at most 8 and 256 MiB in all, the largest released first), so staging per table does not
 * page-lock anew.  *out = NULL for bytes == 0.  Free with
 * pdb_host_free (NULL is a no-op; any other pointer not from pdb_host_alloc: PDB_EINVAL). */
int pdb_host_alloc(uint64_t bytes, void** out);
int pdb_host_free(void* p);

/* ---- host batches (copy-inclusive: H2D + kernel + D2H on the internal stream) ---------------
 * Staged in groups of at most 256 MiB of span, so the device workspace stays bounded. */
int pdb_crc32c_batch_host(const void* base, uint64_t base_len, const pdb_blk* blk, uint64_t nblk,
                          uint32_t flags, uint32_t* out);
/* ReadBlock's check for host blocks: ok[i] = (crc_i == expected[i]) (expected masked iff
 * PDB_CRC_MASK_OUTPUT; ok may be NULL).  Returns the number of mismatches or a negative error. */
int64_t pdb_crc32c_verify_host(const void* base, uint64_t base_len, const pdb_blk* blk, uint64_t nblk,
                               uint32_t flags, const uint32_t* expected, uint8_t* ok);

/* ---- sstable block trailers (table/table_builder.cc:187-205, table/format.cc:66-104) ---------
 * `buf` holds an sstable image (or any span of one) in which each handle's block is followed by
 * its trailer at buf[offset+size .. offset+size+5).  The type byte buf[offset+size] is input. */
/* Seal: write Mask(crc32c(contents||type)) little-endian at buf[offset+size+1]. */
int pdb_sst_seal_device(void* d_buf, uint64_t buf_len, const pdb_block_handle* d_h, uint64_t n,
                        void* stream);
int pdb_sst_seal_host(void* buf, uint64_t buf_len, const pdb_block_handle* h, uint64_t n);
/* The seal's trailer words without writing them: d_out[i] = Mask(crc32c(contents||type)) (the
 * value WriteRawBlock encodes at offset+size+1), for an engine that writes the trailer while it
 * copies blocks out -- the in-place seal pays for scattered 4-B writes, this form does not.  A
 * handle whose block + trailer leaves the image leaves d_out[i] untouched. */
int pdb_sst_crc_device(const void* d_buf, uint64_t buf_len, const pdb_block_handle* d_h, uint64_t n,
                       uint32_t* d_out, void* stream);
/* Verify: ok[i] = 1 iff Unmask(DecodeFixed32(trailer+1)) == crc32c(contents||type).
 * Returns the number of mismatching blocks (>= 0) or a negative error. */
int64_t pdb_sst_verify_host(const void* buf, uint64_t buf_len, const pdb_block_handle* h, uint64_t n,
                            uint8_t* ok);
int pdb_sst_verify_device(const void* d_buf, uint64_t buf_len, const pdb_block_handle* d_h,
                          uint64_t n, uint8_t* d_ok, uint32_t* d_nbad, void* stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* PDB_CRC32C_H_ */
