// diag_capi.cpp -- C-ABI of the bench / test infrastructure library (include/pdb_crc32c_diag.h).
// Per-device tables of its own (no state shared with the product library); every variant is an
// argument, never a global.
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/pdb_crc32c_diag.h"
#include "crc32c_internal.h"
#include "crc32c_math.h"
#include "diag_internal.h"

namespace pdb {
namespace {

thread_local std::string g_diag_err;

int dfail(int code, const std::string& msg) {
  g_diag_err = msg;
  return code;
}

struct DiagDev {
  uint32_t* d_tables = nullptr;
  LaunchGeom geom{256, 1024};
};

std::mutex g_mu;
DiagDev g_devs[64];

int diag_state(const DiagDev** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return dfail(PDB_ENODEV, std::string("hipGetDevice: ") + hipGetErrorString(e));
  if (dev < 0 || dev >= 64) return dfail(PDB_ENODEV, "device index out of range");
  std::lock_guard<std::mutex> lk(g_mu);
  DiagDev& d = g_devs[dev];
  if (!d.d_tables) {
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, dev)) != hipSuccess)
      return dfail(PDB_EHIP, std::string("hipGetDeviceProperties: ") + hipGetErrorString(e));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return dfail(PDB_ENODEV, "built for gfx950 only");
    d.geom.grid = prop.multiProcessorCount > 0 ? static_cast<uint32_t>(prop.multiProcessorCount) : 256;
    std::vector<uint32_t> tabs(PDB_TABLE_WORDS);
    build_device_tables(tabs.data());
    uint32_t* p = nullptr;
    if ((e = hipMalloc(&p, tabs.size() * 4)) != hipSuccess)
      return dfail(PDB_ENOMEM, std::string("hipMalloc(tables): ") + hipGetErrorString(e));
    if ((e = hipMemcpy(p, tabs.data(), tabs.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
      return dfail(PDB_EHIP, std::string("hipMemcpy(tables): ") + hipGetErrorString(e));
    d.d_tables = p;
  }
  *out = &d;
  return PDB_OK;
}

int done(hipError_t e, const char* what) {
  return e == hipSuccess ? PDB_OK : dfail(PDB_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace
}  // namespace pdb

using namespace pdb;

extern "C" {

const char* pdb_diag_last_error(void) { return g_diag_err.c_str(); }

int pdb_diag_fill_splitmix(void* d_dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset, void* stream) {
  if (nbytes && !d_dst) return dfail(PDB_EINVAL, "null argument");
  return done(launch_fill_splitmix(static_cast<uint8_t*>(d_dst), nbytes, seed, byte_offset,
                                   static_cast<hipStream_t>(stream)),
              "fill_splitmix");
}

int pdb_diag_read_stream(const void* d_base, uint64_t nbytes, uint32_t* d_out, void* stream) {
  return done(launch_read_stream(static_cast<const uint8_t*>(d_base), nbytes, d_out, static_cast<hipStream_t>(stream)),
              "read_stream");
}

int pdb_diag_read_pattern4k(const void* d_base, uint64_t nblk, int variant, uint32_t* d_out, void* stream) {
  const DiagDev* d;
  int rc = diag_state(&d);
  if (rc) return rc;
  return done(launch_read_pattern4k(d->geom, static_cast<const uint8_t*>(d_base), nblk, variant, d_out,
                                    static_cast<hipStream_t>(stream)),
              "read_pattern4k");
}

int pdb_diag_batch_fixed(int variant, const void* d_base, uint64_t stride, uint32_t len, uint64_t nblk,
                         uint32_t flags, uint32_t init, uint32_t* d_out, void* stream) {
  if (nblk == 0) return PDB_OK;
  if (!d_base || !d_out) return dfail(PDB_EINVAL, "null argument");
  const DiagDev* d;
  int rc = diag_state(&d);
  if (rc) return rc;
  return done(launch_fixed_variant(variant, d->geom, d->d_tables, static_cast<const uint8_t*>(d_base), stride, len,
                                   nblk, flags, init, d_out, static_cast<hipStream_t>(stream)),
              "batch_fixed variant");
}

int pdb_diag_batch_desc(int variant, const void* d_base, const pdb_blk* d_blk, uint64_t nblk, uint32_t flags,
                        uint32_t* d_out, void* stream) {
  if (nblk == 0) return PDB_OK;
  if (!d_base || !d_blk || !d_out) return dfail(PDB_EINVAL, "null argument");
  const DiagDev* d;
  int rc = diag_state(&d);
  if (rc) return rc;
  return done(launch_desc_variant(variant, d->geom, d->d_tables, static_cast<const uint8_t*>(d_base), d_blk, nblk,
                                  flags, d_out, static_cast<hipStream_t>(stream)),
              "batch_desc variant");
}

int pdb_diag_sst(int variant, void* d_buf, uint64_t buf_len, const pdb_block_handle* d_h, uint64_t n, int seal,
                 uint8_t* d_ok, uint32_t* d_nbad, void* stream) {
  if (n == 0) return PDB_OK;
  if (!d_buf || !d_h) return dfail(PDB_EINVAL, "null argument");
  if (buf_len < 5) return dfail(PDB_ERANGE, "buffer smaller than one block trailer");
  const DiagDev* d;
  int rc = diag_state(&d);
  if (rc) return rc;
  return done(launch_sst_variant(variant, d->geom, d->d_tables, static_cast<uint8_t*>(d_buf), buf_len, d_h, n,
                                 seal != 0, d_ok, d_nbad, static_cast<hipStream_t>(stream)),
              "sst variant");
}

}  // extern "C"
