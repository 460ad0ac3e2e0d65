// crc32c_capi.cpp -- the C-ABI boundary (include/pdb_crc32c.h) over the HIP kernels.
//
// Replaces leveldb::crc32c::{Extend,Value,Mask,Unmask} (reference util/crc32c.h:14-40) and the
// trailer math inside TableBuilder::WriteRawBlock / ReadBlock (table/table_builder.cc:187-205,
// table/format.cc:96-104).  There is deliberately no CPU implementation of the CRC here: every
// checksum is computed by the gfx950 kernels, and a missing device is an error.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sched.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "crc32c_internal.h"
#include "crc32c_math.h"

namespace pdb {

LongLane long_lane_at(uint8_t* d, const uint32_t* d_pow2) {
  LongLane ll{};
  if (!d) return ll;
  ll.hdr = reinterpret_cast<unsigned long long*>(d);
  ll.rec = reinterpret_cast<LongRec*>(d + kLongRecOff);
  ll.piece = reinterpret_cast<LongPiece*>(d + kLongPieceOff);
  ll.leaf = reinterpret_cast<uint32_t*>(d + kLongLeafOff);
  ll.pow2 = d_pow2;
  ll.rec_cap = kLongRecCap;
  ll.piece_cap = kLongPieceCap;
  return ll;
}

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(PDB_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// A host-staging context: streams, pipeline events and a device workspace.  Host batches from
// different threads (the engine's compaction seals, scan windows, log checks) take different
// contexts and run concurrently instead of queueing on one device mutex.
struct HostCtx {
  std::mutex mu;
  hipStream_t stream = nullptr;       // kernels and result copies of the host entry points
  hipStream_t copy_stream = nullptr;  // host -> device staging copies (overlap the previous group's kernel)
  hipEvent_t staged[2] = {};          // group in workspace slot k copied in
  hipEvent_t drained[2] = {};         // group in workspace slot k hashed and its results copied out
  uint8_t* d_ws = nullptr;
  size_t ws_cap = 0;
  // page-locked host scratch for a call's small per-block arrays (rebased handles in, trailer words
  // / ok bytes out): DMA'd directly instead of through the runtime's pageable bounce buffers
  uint8_t* h_pin = nullptr;
  uint8_t* d_pin = nullptr;  // its device mapping (the zero-copy sst path's handles and ok bytes)
  size_t h_pin_cap = 0;
  uint8_t* d_lane = nullptr;  // long-block lane scratch (long_scratch_bytes(), made at the first long block)
};
constexpr int kHostCtx = 4;

// One scalar-service request slot (crc32c_server.hip): its request sequence number, guarded by mu
// (a slot is shared only when more threads than slots call at once).
struct ScalarSlot {
  std::mutex mu;
  uint32_t seq = 0;
};

struct DevState {
  int device = -1;
  uint32_t* d_tables = nullptr;
  uint32_t* d_pow2 = nullptr;  // 64 power-of-two shift operators (long-span combine)
  LaunchGeom geom{256, 1024};
  // host entry points: one CU is left to the scalar service, so a host batch never has to stop it
  // (a batch's persistent workgroups need a whole CU each) and scalar calls keep being answered
  // while batches run
  LaunchGeom hgeom{255, 1024};
  HostCtx ctx[kHostCtx];
  std::mutex mu;  // the launch-per-call scalar modes' staging below
  // scalar Extend: pinned, device-mapped staging ([256-B result area][bytes]); the kernels read
  // the bytes across PCIe and write the CRC back into it, so a call is memcpy + launch(es) + sync
  uint8_t* h_stage = nullptr;
  uint8_t* d_stage = nullptr;  // device alias of h_stage
  size_t stage_cap = 0;
  uint32_t seq = 0;          // scalar-call sentinel sequence
  // kScalarPoll returns when the result word lands, before its kernel has ended (and the next call
  // may take another context's stream): an event after every such launch, waited on before the
  // stage is freed or regrown
  hipEvent_t stage_done = nullptr;
  bool stage_pending = false;
  // Scalar calls <= kServerCap: kScalarServer (default) posts them to the persistent server
  // kernel (crc32c_server.hip); PDB_SCALAR_WAIT=poll launches one kernel per call and spins on
  // the result, =sync waits on the stream (A/B diagnostics, tools/scalar_latency.py).
  int scalar_mode = 0;
  std::mutex srv_mu;             // server allocation, launch and stop (never held across a request)
  uint8_t* srv_in_h = nullptr;   // request area (kServerInBytes), host-writable address
  uint8_t* srv_in_d = nullptr;   // its device address
  bool srv_in_device = false;    // request area in fine-grained device memory (large BAR)
  uint8_t* srv_out_h = nullptr;  // response area (kServerOutBytes, pinned host memory)
  uint8_t* srv_out_d = nullptr;
  bool large_bar = false;
  hipStream_t srv_stream = nullptr;
  uint32_t srv_epoch = 0;        // epoch of the most recently launched server (atomic)
  uint64_t srv_stop = 0;         // ctl->stop value the live instance runs under (srv_mu)
  bool srv_live = false;         // an instance of srv_epoch may still be in its loop (atomic)
  ScalarSlot slots[kServerSlots];
  // PDB_SERVER_STAMPS=<path> (diagnostics, tools/scalar_phases.py): every scalar call records its host
  // clock at entry, after posting and on seeing the answer, and the server's poll / hash-done ticks;
  // the rows are written to <path> at exit
  bool stamps = false;
  // the long-block lane of device-resident calls, one scratch per caller stream (made at the stream's
  // first call outside a capture, or by pdb_crc32c_prepare_stream; kept for the process)
  std::mutex lane_mu;
  std::vector<std::pair<hipStream_t, uint8_t*>> lanes;
};
constexpr size_t kMaxStreamLanes = 64;

struct PhaseStamp {
  uint64_t n, h0, h1, h2, g_seen, g_done;  // bytes; host CLOCK_MONOTONIC ns; s_memrealtime ticks
};
std::mutex g_stamp_mu;
std::vector<PhaseStamp> g_stamps;

// PDB_SEAL_STAMPS=<path> (diagnostics): every zero-copy host seal / verify records its bytes, its
// host clock at entry, with its context locked, after the launch and after the synchronisation,
// and the kernel's own time (events around it); the rows are written to <path> at exit
struct SealStamp {
  uint64_t n, t0, t1, t2, t3, allocs, nblk, maxblk;  // allocs: pdb_host_alloc page-locking calls so far
  float kern_ms;
};
std::atomic<uint64_t> g_pin_allocs{0};
std::mutex g_seal_stamp_mu;
std::vector<SealStamp> g_seal_stamps;
void write_seal_stamps_at_exit() {
  const char* path = getenv("PDB_SEAL_STAMPS");
  if (!path) return;
  std::lock_guard<std::mutex> lk(g_seal_stamp_mu);
  FILE* f = fopen(path, "w");
  if (!f) return;
  fprintf(f, "bytes,entry_ns,locked_ns,launched_ns,synced_ns,kernel_ms,allocs,blocks,max_block\n");
  for (const SealStamp& p : g_seal_stamps)
    fprintf(f, "%llu,%llu,%llu,%llu,%llu,%.4f,%llu,%llu,%llu\n", (unsigned long long)p.n, (unsigned long long)p.t0,
            (unsigned long long)p.t1, (unsigned long long)p.t2, (unsigned long long)p.t3, p.kern_ms,
            (unsigned long long)p.allocs, (unsigned long long)p.nblk, (unsigned long long)p.maxblk);
  fclose(f);
}
bool seal_stamps_on() {
  static const bool v = [] {
    if (!getenv("PDB_SEAL_STAMPS")) return false;
    atexit(write_seal_stamps_at_exit);
    return true;
  }();
  return v;
}

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<uint64_t>(ts.tv_sec) * 1000000000ull + static_cast<uint64_t>(ts.tv_nsec);
}

void write_stamps_at_exit() {
  const char* path = getenv("PDB_SERVER_STAMPS");
  if (!path) return;
  std::lock_guard<std::mutex> lk(g_stamp_mu);
  FILE* f = fopen(path, "w");
  if (!f) return;
  fprintf(f, "n,h0_ns,h1_ns,h2_ns,g_seen_tick,g_done_tick\n");
  for (const PhaseStamp& p : g_stamps)
    fprintf(f, "%llu,%llu,%llu,%llu,%llu,%llu\n", (unsigned long long)p.n, (unsigned long long)p.h0,
            (unsigned long long)p.h1, (unsigned long long)p.h2, (unsigned long long)p.g_seen,
            (unsigned long long)p.g_done);
  fclose(f);
}

enum ScalarMode : int { kScalarServer = 0, kScalarPoll = 1, kScalarSync = 2 };
// Server lifetime (s_memrealtime ticks, 100 MHz): it leaves after 20 ms without a request or
// 200 ms in total; the next call relaunches it (~20 us), so a process that dies or forgets to stop
// it never leaves a kernel spinning for long.
constexpr uint64_t kServerIdleTicks = 2000000ull;
constexpr uint64_t kServerLifeTicks = 20000000ull;

constexpr int kMaxDev = 64;
std::mutex g_init_mu;
DevState* g_dev[kMaxDev] = {};

int get_state(DevState** out) {
  int dev = 0;
  static int g_ndev = 0;  // device count, cached once positive
  if (__atomic_load_n(&g_ndev, __ATOMIC_ACQUIRE) <= 0) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0)
      return fail(PDB_ENODEV, "no HIP device visible (pdb_crc32c has no CPU fallback)");
    __atomic_store_n(&g_ndev, n, __ATOMIC_RELEASE);
  }
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  if (dev < 0 || dev >= kMaxDev) return fail(PDB_ENODEV, "device index out of range");
  DevState* st = __atomic_load_n(&g_dev[dev], __ATOMIC_ACQUIRE);
  if (st) {
    *out = st;
    return PDB_OK;
  }
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (g_dev[dev]) {
    *out = g_dev[dev];
    return PDB_OK;
  }
  std::unique_ptr<DevState> s(new DevState);
  s->device = dev;
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(PDB_ENODEV, std::string("pdb_crc32c is built for gfx950; device is ") +
                                prop.gcnArchName);
  s->geom.grid = prop.multiProcessorCount > 0 ? static_cast<uint32_t>(prop.multiProcessorCount) : 256;
  s->geom.block = 1024;
  s->large_bar = prop.isLargeBar != 0;
  std::vector<uint32_t> tabs(PDB_TABLE_WORDS);
  build_device_tables(tabs.data());
  e = hipMalloc(&s->d_tables, tabs.size() * sizeof(uint32_t));
  if (e != hipSuccess) return hip_fail(e, "hipMalloc(tables)");
  e = hipMemcpy(s->d_tables, tabs.data(), tabs.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, "hipMemcpy(tables)");
  std::vector<uint32_t> pow2(PDB_POW2_WORDS);
  build_pow2_tables(pow2.data());
  e = hipMalloc(&s->d_pow2, pow2.size() * sizeof(uint32_t));
  if (e != hipSuccess) return hip_fail(e, "hipMalloc(pow2)");
  e = hipMemcpy(s->d_pow2, pow2.data(), pow2.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, "hipMemcpy(pow2)");
  const char* wait = getenv("PDB_SCALAR_WAIT");
  s->scalar_mode = !wait ? kScalarServer
                          : strcmp(wait, "sync") == 0 ? kScalarSync
                          : strcmp(wait, "poll") == 0 ? kScalarPoll : kScalarServer;
  s->hgeom.grid = s->geom.grid > 1 ? s->geom.grid - 1 : 1;
  s->stamps = getenv("PDB_SERVER_STAMPS") != nullptr;
  if (s->stamps) {
    static std::once_flag once;
    std::call_once(once, [] { atexit(write_stamps_at_exit); });
  }
  for (HostCtx& c : s->ctx) {
    e = hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail(e, "hipStreamCreate");
    e = hipStreamCreateWithFlags(&c.copy_stream, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail(e, "hipStreamCreate(copy)");
    for (int k = 0; k < 2; ++k) {
      if ((e = hipEventCreateWithFlags(&c.staged[k], hipEventDisableTiming)) != hipSuccess ||
          (e = hipEventCreateWithFlags(&c.drained[k], hipEventDisableTiming)) != hipSuccess)
        return hip_fail(e, "hipEventCreate");
    }
  }
  __atomic_store_n(&g_dev[dev], s.get(), __ATOMIC_RELEASE);
  *out = s.release();
  return PDB_OK;
}

// Device entry points launch on the caller's stream; NULL is the HIP default (null) stream,
// exactly as for hipMemcpyAsync/hipLaunchKernel (torch's default stream is that stream).
hipStream_t pick_stream(DevState* st, void* stream) {
  (void)st;
  return static_cast<hipStream_t>(stream);
}

// A zeroed long-block lane scratch, ordered before the first use on stream s.
int alloc_lane(hipStream_t s, uint8_t** out) {
  void* d = nullptr;
  hipError_t e = hipMalloc(&d, long_scratch_bytes());
  if (e != hipSuccess) return fail(PDB_ENOMEM, std::string("hipMalloc(long-block lane): ") + hipGetErrorString(e));
  if ((e = hipMemsetAsync(d, 0, kLongHdrBytes, s)) != hipSuccess) {
    (void)hipFree(d);
    return hip_fail(e, "hipMemsetAsync(long-block lane)");
  }
  *out = static_cast<uint8_t*>(d);
  return PDB_OK;
}

// The long-block lane for device-resident calls on `s` (crc32c_internal.h): the stream's own scratch,
// made at its first call.  Inside a stream capture nothing is allocated: a stream that was never
// prepared (pdb_crc32c_prepare_stream) then runs without the lane -- long blocks are hashed by the
// batch kernel's one-wave path, with identical results.  Past kMaxStreamLanes streams, likewise.
const LongLane* stream_lane(DevState* st, hipStream_t s, LongLane* ll, bool may_alloc = true) {
  std::lock_guard<std::mutex> lk(st->lane_mu);
  for (const auto& x : st->lanes)
    if (x.first == s) {
      *ll = long_lane_at(x.second, st->d_pow2);
      return ll;
    }
  if (!may_alloc || st->lanes.size() >= kMaxStreamLanes) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  uint8_t* d = nullptr;
  if (alloc_lane(s, &d)) return nullptr;
  st->lanes.emplace_back(s, d);
  *ll = long_lane_at(d, st->d_pow2);
  return ll;
}

int ensure_ws(HostCtx* c, size_t bytes) {
  if (bytes <= c->ws_cap) return PDB_OK;
  if (c->d_ws) {
    (void)hipStreamSynchronize(c->copy_stream);
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->d_ws);
    c->d_ws = nullptr;
    c->ws_cap = 0;
  }
  size_t cap = std::max<size_t>(bytes, 1 << 20);
  hipError_t e = hipMalloc(&c->d_ws, cap);
  if (e != hipSuccess) return fail(PDB_ENOMEM, std::string("hipMalloc(workspace): ") + hipGetErrorString(e));
  c->ws_cap = cap;
  return PDB_OK;
}

int ensure_pin(HostCtx* c, size_t bytes) {
  if (bytes <= c->h_pin_cap) return PDB_OK;
  if (c->h_pin) {
    (void)hipStreamSynchronize(c->copy_stream);
    (void)hipStreamSynchronize(c->stream);
    (void)hipHostFree(c->h_pin);
    c->h_pin = nullptr;
    c->h_pin_cap = 0;
  }
  size_t cap = std::max<size_t>(bytes, 1 << 16);
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&c->h_pin), cap, hipHostMallocDefault);
  if (e != hipSuccess) return fail(PDB_ENOMEM, std::string("hipHostMalloc(scratch): ") + hipGetErrorString(e));
  c->h_pin_cap = cap;
  void* d = nullptr;
  c->d_pin = hipHostGetDevicePointer(&d, c->h_pin, 0) == hipSuccess ? static_cast<uint8_t*>(d) : nullptr;
  return PDB_OK;
}

// pdb_host_alloc's allocations: page-locked, with their device mappings.  A freed one is kept for
// reuse (a TableBuilder stages every table in a fresh buffer; page-locking megabytes per table costs
// more than the seal), at most kPinKeep of them and kPinKeepBytes in all: past either, the largest
// kept ones are released first.
struct PinAlloc {
  uint8_t* h;
  uint8_t* d;  // device mapping (null: none)
  size_t cap;
  bool used;
};
std::mutex g_pin_mu;
std::vector<PinAlloc> g_pins;
constexpr size_t kPinKeep = 8;
constexpr size_t kPinKeepBytes = size_t(256) << 20;

// The device mapping of [p, p + len) when it lies inside one live pdb_host_alloc allocation, else null.
uint8_t* pin_mapping(const void* p, uint64_t len) {
  const uint8_t* q = static_cast<const uint8_t*>(p);
  std::lock_guard<std::mutex> lk(g_pin_mu);
  for (const PinAlloc& a : g_pins)
    if (a.used && a.d && q >= a.h && len <= a.cap && static_cast<size_t>(q - a.h) <= a.cap - len) return a.d + (q - a.h);
  return nullptr;
}

// A free host context (try each once), else the one this thread hashes to.
struct CtxLock {
  HostCtx* c;
  std::unique_lock<std::mutex> lk;
  explicit CtxLock(DevState* st) : c(nullptr) {
    for (HostCtx& x : st->ctx) {
      std::unique_lock<std::mutex> t(x.mu, std::try_to_lock);
      if (t.owns_lock()) {
        c = &x;
        lk = std::move(t);
        return;
      }
    }
    static std::atomic<uint32_t> rr{0};
    thread_local uint32_t mine = rr.fetch_add(1, std::memory_order_relaxed);
    c = &st->ctx[mine % kHostCtx];
    lk = std::unique_lock<std::mutex>(c->mu);
  }
};

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

constexpr size_t kStageHdr = 256;  // result words ahead of the staged bytes (keeps them 256-B aligned)

int ensure_stage(DevState* st, size_t bytes) {
  if (bytes <= st->stage_cap) return PDB_OK;
  if (st->h_stage) {  // (st->mu held: every user of the stage has synchronised its stream, or --
                      // a poll-mode call that returned early -- recorded stage_done after its kernel)
    if (st->stage_pending) {
      (void)hipEventSynchronize(st->stage_done);
      st->stage_pending = false;
    }
    (void)hipHostFree(st->h_stage);
    st->h_stage = st->d_stage = nullptr;
    st->stage_cap = 0;
  }
  size_t cap = std::max<size_t>(bytes, 64 << 10);
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&st->h_stage), cap,
                               hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return fail(PDB_ENOMEM, std::string("hipHostMalloc(stage): ") + hipGetErrorString(e));
  void* dp = nullptr;
  if ((e = hipHostGetDevicePointer(&dp, st->h_stage, 0)) != hipSuccess) {
    (void)hipHostFree(st->h_stage);
    st->h_stage = nullptr;
    return hip_fail(e, "hipHostGetDevicePointer(stage)");
  }
  st->d_stage = static_cast<uint8_t*>(dp);
  st->stage_cap = cap;
  return PDB_OK;
}

// ---- scalar Extend service (crc32c_server.hip) -------------------------------------------------
double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

uint32_t box_load(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

ServerCtl* srv_ctl(const DevState* st) { return reinterpret_cast<ServerCtl*>(st->srv_in_h); }
uint64_t* srv_req(const DevState* st, uint32_t slot) {
  return reinterpret_cast<uint64_t*>(st->srv_in_h + kReqOff) + slot;
}
uint8_t* srv_data(const DevState* st, uint32_t slot) { return st->srv_in_h + kSlotDataOff + slot * kSlotStride; }
const uint64_t* srv_resp(const DevState* st, uint32_t slot) {
  return reinterpret_cast<const uint64_t*>(st->srv_out_h + 64u * slot);
}
ServerExit* srv_exit(const DevState* st) { return reinterpret_cast<ServerExit*>(st->srv_out_h + kExitOff); }

uint32_t live_epoch(const DevState* st) { return __atomic_load_n(&st->srv_epoch, __ATOMIC_ACQUIRE); }
bool server_exited(const DevState* st, uint32_t epoch) { return box_load(&srv_exit(st)->exit_epoch) == epoch; }

// The request box may be device memory written through the BAR (write-combined): the fences order
// the staged bytes before the request word and push the word out at once.
void post_word(uint64_t* p, uint64_t w) {
  __builtin_ia32_sfence();
  __atomic_store_n(p, w, __ATOMIC_RELEASE);
  __builtin_ia32_sfence();
}

// Ask the live instance to leave and wait until it has (srv_mu held).  Host memory only, no HIP
// call, so it is safe inside stream capture.  Every wave polls ctl->stop (~2 us); the lifetime
// bounds the wait in any case.
int server_park(DevState* st) {
  if (!__atomic_load_n(&st->srv_live, __ATOMIC_ACQUIRE)) return PDB_OK;
  const uint32_t epoch = live_epoch(st);
  if (!server_exited(st, epoch)) {
    post_word(&srv_ctl(st)->stop, ++st->srv_stop);
    const double t0 = now_s();
    while (!server_exited(st, epoch)) {
      __builtin_ia32_pause();
      if (now_s() - t0 > 2.0) return fail(PDB_EHIP, "scalar server did not stop within 2 s");
    }
  }
  __atomic_store_n(&st->srv_live, false, __ATOMIC_RELEASE);
  return PDB_OK;
}

// Device-resident batches launch a workgroup on every CU: stop a live server first (host batches
// leave it a CU instead, DevState::hgeom).
int quiesce(DevState* st) {
  if (!__atomic_load_n(&st->srv_live, __ATOMIC_ACQUIRE)) return PDB_OK;
  std::lock_guard<std::mutex> lk(st->srv_mu);
  return server_park(st);
}

void park_all_at_exit() {
  for (int d = 0; d < kMaxDev; ++d) {
    DevState* st = __atomic_load_n(&g_dev[d], __ATOMIC_ACQUIRE);
    if (!st || !__atomic_load_n(&st->srv_live, __ATOMIC_ACQUIRE)) continue;
    std::unique_lock<std::mutex> lk(st->srv_mu, std::try_to_lock);
    if (!lk.owns_lock()) continue;  // a launch in flight at exit: the idle timeout ends the server
    const uint32_t epoch = live_epoch(st);
    if (!server_exited(st, epoch)) post_word(&srv_ctl(st)->stop, ++st->srv_stop);
    const double t0 = now_s();
    while (!server_exited(st, epoch) && now_s() - t0 < 0.5) __builtin_ia32_pause();
  }
}

int alloc_pinned(size_t bytes, uint8_t** h, uint8_t** d) {
  void* hp = nullptr;
  hipError_t e = hipHostMalloc(&hp, bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return fail(PDB_ENOMEM, std::string("hipHostMalloc(server): ") + hipGetErrorString(e));
  memset(hp, 0, bytes);
  void* dp = nullptr;
  if ((e = hipHostGetDevicePointer(&dp, hp, 0)) != hipSuccess) {
    (void)hipHostFree(hp);
    return hip_fail(e, "hipHostGetDevicePointer(server)");
  }
  *h = static_cast<uint8_t*>(hp);
  *d = static_cast<uint8_t*>(dp);
  return PDB_OK;
}

// (srv_mu held)
int server_alloc(DevState* st) {
  hipError_t e;
  int rc;
  // request area: fine-grained device memory written by the host through the large BAR (the
  // server polls local HBM: ~0.37 us per poll vs ~1.2 us across PCIe, tools/server_probe.hip), else
  // pinned host memory.  PDB_SERVER_BOX=host forces the latter (A/B).
  const char* where = getenv("PDB_SERVER_BOX");
  const bool want_dev = st->large_bar && !(where && strcmp(where, "host") == 0);
  if (want_dev) {
    void* p = nullptr;
    e = hipExtMallocWithFlags(&p, kServerInBytes, hipDeviceMallocFinegrained);
    if (e == hipSuccess) {
      if ((e = hipMemset(p, 0, kServerInBytes)) != hipSuccess) return hip_fail(e, "hipMemset(server box)");
      if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(e, "hipDeviceSynchronize(server box)");
      st->srv_in_h = st->srv_in_d = static_cast<uint8_t*>(p);
      st->srv_in_device = true;
    }
  }
  if (!st->srv_in_h && (rc = alloc_pinned(kServerInBytes, &st->srv_in_h, &st->srv_in_d))) return rc;
  if ((rc = alloc_pinned(kServerOutBytes, &st->srv_out_h, &st->srv_out_d))) return rc;
  // The server's stream gets the greatest priority: the runtime keeps a separate hardware-queue
  // pool per priority, so no host-context stream (normal priority; 8 of them over
  // GPU_MAX_HW_QUEUES = 4 queues) shares the server's queue.  On a shared queue a host batch's
  // kernel would sit behind the persistent server for up to its 200-ms lifetime (ADVICE r03;
  // tests/test_scalar_server.py::test_scalar_callers_beside_batch_seals times every batch).
  int prio_least = 0, prio_greatest = 0;
  if ((e = hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest)) != hipSuccess)
    return hip_fail(e, "hipDeviceGetStreamPriorityRange");
  if ((e = hipStreamCreateWithPriority(&st->srv_stream, hipStreamNonBlocking, prio_greatest)) != hipSuccess)
    return hip_fail(e, "hipStreamCreate(server)");
  static std::once_flag once;
  std::call_once(once, [] { atexit(park_all_at_exit); });
  return PDB_OK;
}

// Make sure an instance is serving (or about to): launch one if none is live, or if the instance
// `seen` (the epoch the caller observed) has left.  srv_mu serialises launches; a thread that
// finds the epoch already bumped by another caller just goes on waiting for its answer.
int server_ensure(DevState* st, bool relaunch_seen, uint32_t seen) {
  std::lock_guard<std::mutex> lk(st->srv_mu);
  int rc;
  if (!st->srv_stream && (rc = server_alloc(st))) return rc;
  const bool live = __atomic_load_n(&st->srv_live, __ATOMIC_ACQUIRE);
  const uint32_t epoch = live_epoch(st);
  if (live && !server_exited(st, epoch)) return PDB_OK;            // serving
  if (relaunch_seen && live && epoch != seen) return PDB_OK;        // another caller relaunched it
  hipError_t e = hipSetDevice(st->device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  const uint32_t next = epoch + 1;
  e = launch_server(st->d_tables, st->srv_in_d, st->srv_out_d, next, st->srv_stop, kServerIdleTicks, kServerLifeTicks,
                    st->stamps ? 1u : 0u, st->srv_stream);
  if (e != hipSuccess) return hip_fail(e, "launch_server");
  __atomic_store_n(&st->srv_epoch, next, __ATOMIC_RELEASE);
  __atomic_store_n(&st->srv_live, true, __ATOMIC_RELEASE);
  return PDB_OK;
}

// This thread's request slot: assigned round robin at the thread's first call.
uint32_t my_slot() {
  static std::atomic<uint32_t> next{0};
  thread_local uint32_t slot = next.fetch_add(1, std::memory_order_relaxed) % kServerSlots;
  return slot;
}

// Scalar waiters of this process (server_call's wait loop) and the CPUs it may run on: the affinity
// mask, capped by a cgroup v2 CPU quota when one is set (a container's nproc shows the host's CPUs).
std::atomic<uint32_t> g_waiters{0};
struct WaitGuard {
  WaitGuard() { g_waiters.fetch_add(1, std::memory_order_relaxed); }
  ~WaitGuard() { g_waiters.fetch_sub(1, std::memory_order_relaxed); }
};
uint32_t wait_cpus() {
  static const uint32_t v = [] {
    cpu_set_t set;
    uint32_t n = sched_getaffinity(0, sizeof(set), &set) == 0 ? static_cast<uint32_t>(CPU_COUNT(&set)) : 1u;
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char quota[32];
      unsigned long long period = 0;
      if (fscanf(f, "%31s %llu", quota, &period) == 2 && strcmp(quota, "max") != 0 && period) {
        const unsigned long long c = (strtoull(quota, nullptr, 10) + period - 1) / period;
        if (c && c < n) n = static_cast<uint32_t>(c);
      }
      fclose(f);
    }
    return n ? n : 1u;
  }();
  return v;
}

// One request (n <= kServerCap) in this thread's slot: stage the bytes, post the request word,
// spin on the slot's response word.  No device-wide lock: other threads' requests proceed in
// their own slots.  An instance that left without answering (idle / lifetime exit racing the
// post) is replaced; the new one serves every pending slot.
int server_call(DevState* st, uint32_t init, const uint8_t* data, uint64_t n, uint32_t* out) {
  int rc;
  const uint32_t slot = my_slot();
  ScalarSlot& sl = st->slots[slot];
  std::lock_guard<std::mutex> lk(sl.mu);
  if (!__atomic_load_n(&st->srv_live, __ATOMIC_ACQUIRE) || server_exited(st, live_epoch(st)))
    if ((rc = server_ensure(st, false, 0))) return rc;
  const uint64_t h0 = st->stamps ? mono_ns() : 0;
  memcpy(srv_data(st, slot) + ((0u - static_cast<uint32_t>(n)) & 15u), data, n);
  const uint32_t seq = sl.seq = (sl.seq + 1) & kServerSeqMask;
  post_word(srv_req(st, slot), (static_cast<uint64_t>((seq << 17) | static_cast<uint32_t>(n)) << 32) | init);
  const uint64_t h1 = st->stamps ? mono_ns() : 0;
  const uint64_t* resp = srv_resp(st, slot);
  double t0 = 0;
  // Wait: spin (pause) while this process has no more waiters than CPUs, else give the CPU back between
  // polls (sched_yield).  A verified point read waits ~5 us for its answer; spinning is the cheapest
  // wait while every waiter has a CPU (8 / 16 reader threads on a 16-CPU box: 560 k / 612 k reads/s
  // spinning against 369 k / 393 k yielding after 2 us), and only with more waiters than CPUs do the
  // spinners take the CPU the others need (32 threads: 246 k spinning, 369 k yielding).  This form, on
  // one box: 551 / 684 / 498 / 404 k reads/s at 8 / 16 / 24 / 32 threads against 453 / 506 / 407 / 286
  // k always spinning -- profiles/r06/point_reads, DESIGN.md §8, INTEGRATION.md §3.
  WaitGuard wg;
  const uint32_t cpus = wait_cpus();
  for (uint32_t spin = 1;; ++spin) {
    const uint64_t r = __atomic_load_n(resp, __ATOMIC_ACQUIRE);
    if (static_cast<uint32_t>(r >> 32) == seq) {
      *out = static_cast<uint32_t>(r);
      if (st->stamps) {
        const uint64_t h2 = mono_ns();
        const PhaseStamp ps{n, h0, h1, h2, __atomic_load_n(resp + 1, __ATOMIC_ACQUIRE), __atomic_load_n(resp + 2, __ATOMIC_ACQUIRE)};
        std::lock_guard<std::mutex> lk2(g_stamp_mu);
        g_stamps.push_back(ps);
      }
      return PDB_OK;
    }
    const uint32_t ep = live_epoch(st);
    if (server_exited(st, ep)) {
      // re-check the answer first: the instance may have answered and then left
      if (static_cast<uint32_t>(__atomic_load_n(resp, __ATOMIC_ACQUIRE) >> 32) == seq) continue;
      if ((rc = server_ensure(st, true, ep))) return rc;
    }
    if (g_waiters.load(std::memory_order_relaxed) > cpus) sched_yield();
    else __builtin_ia32_pause();
    if ((spin & 0xFFFFu) == 0) {
      const double t = now_s();
      if (t0 == 0) t0 = t;
      else if (t - t0 > 10.0) return fail(PDB_EHIP, "scalar server gave no answer within 10 s");
    }
  }
}

// Host batches are staged in groups whose byte span is at most host_chunk_bytes() (a block longer than
// that forms its own group), so the device workspace stays bounded however large the host batch.
// Groups alternate between two workspace slots (SlotPipe): group k's host->device copies run on
// copy_stream as soon as slot k & 1 is drained, its kernel and result copy on stream once its copies
// are in -- group k+1's copies overlap group k's kernel and result copy.  One synchronisation at the
// end.  The copies dominate (the kernel is ~1 % of a PCIe copy of the same bytes).
uint64_t host_chunk_bytes() {
  // 256 MiB by default; PDB_HOST_CHUNK_BYTES (read once per process, >= 4 KiB) overrides it for
  // experiments and for tests that exercise multi-group staging on small buffers
  static const uint64_t v = [] {
    const char* e = getenv("PDB_HOST_CHUNK_BYTES");
    const unsigned long long x = e ? strtoull(e, nullptr, 10) : 0ull;
    return x >= 4096ull ? static_cast<uint64_t>(x) : (256ull << 20);
  }();
  return v;
}

// PDB_CRC_SIZE_MIXED for the 512 / 1023 record classes: the record kernel's per-record lanes
// (crc32c_lanespan.h, open_batch) pay when a batch of 64 consecutive records needs fewer items with
// them than with every record on the longest one's lane count; set when a quarter of the batches do
// (a log of equal records with its block-end fragments never does).
static bool mixed_lengths(const pdb_blk* blk, uint64_t nblk, uint32_t cls) {
  const uint32_t part_words = cls == 512u ? 27u : 33u, kmax = cls == 512u ? 5u : 8u;
  uint64_t nb = 0, win = 0;
  for (uint64_t b = 0; b < nblk; b += 64) {
    uint32_t kmx = 0, sumk = 0, nf = 0;
    for (uint64_t i = b; i < nblk && i < b + 64; ++i) {
      const uint32_t len = blk[i].len;
      if (len - 1u > cls - 1u) continue;  // outside the class: the whole-wave path
      const uint32_t k = std::min(kmax, ((len + 3u) / 4u + part_words - 1u) / part_words);
      sumk += k;
      kmx = std::max(kmx, k);
      ++nf;
    }
    if (!nf) continue;
    ++nb;
    const uint32_t g = 64u / kmx;
    if ((sumk + 63u) / 64u < (nf + g - 1u) / g) ++win;
  }
  return nb && 4 * win >= nb;
}

// Records of <= 256 B: the 256 class hashes 33-word parts (k = 1..2 lanes a record, 9 steps an
// item, 11 waves x 8928-B regions), the 512 class 27-word parts (k = 1..5, 8 steps, 12 waves x 8 KiB).
// Records of 133..216 B need two parts in either and the 512 class then runs faster (+17 % on random
// 1-200-B records, tools/ab_hints.py); up to 132 B the 256 class takes one lane a record (wal100),
// past 216 B the 512 class needs three.  A per-batch item count of both decides.
static bool small_records_prefer_512(const pdb_blk* blk, uint64_t nblk) {
  double c256 = 0, c512 = 0;
  for (uint64_t b = 0; b < nblk; b += 64) {
    uint32_t nw = 0, n = 0;
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint64_t i = b; i < nblk && i < b + 64; ++i) {
      const uint32_t len = blk[i].len;
      if (len - 1u > 255u) continue;
      nw = std::max(nw, (len + 3u) / 4u);
      lo = std::min(lo, blk[i].off);
      hi = std::max(hi, blk[i].off + len);
      ++n;
    }
    if (!n) continue;
    const uint64_t span = hi - lo;
    const uint32_t k256 = nw <= 33u ? 1u : 2u, k512 = (nw + 26u) / 27u;
    const uint64_t i256 = std::max<uint64_t>((n + 64u / k256 - 1u) / (64u / k256), (span + 8911u) / 8912u);
    const uint64_t i512 = std::max<uint64_t>((n + 64u / k512 - 1u) / (64u / k512), (span + 8175u) / 8176u);
    c256 += static_cast<double>(i256) * (9 + 4) / 11.0;  // items x (steps + 4) / waves
    c512 += static_cast<double>(i512) * (8 + 4) / 12.0;
  }
  return c512 < 0.95 * c256;
}

// ---- host batches: staging plan, striped over the devices of pdb_crc32c_init_mask ------------------
// A group is a run of consecutive blocks staged by one copy: its span [lo, hi) (lo 16-B aligned down,
// keeping the source's phase so the kernels' fast loads stay aligned) is at most host_chunk_bytes() (a
// longer block forms its own group).  With several devices (pdb_crc32c_init_mask), device d takes a
// contiguous run of groups holding ~1/N of the batch's bytes -- every device stages from its own PCIe
// link at once -- and a batch of less than kStripeMinBytes per device uses fewer devices.
struct HostGroup {
  uint64_t first, count, lo, hi;
  uint32_t dev;  // index into the call's device list
};

std::atomic<uint64_t> g_host_mask{0};  // pdb_crc32c_init_mask (0: the calling thread's device)
constexpr uint64_t kStripeMinBytes = 8ull << 20;

std::vector<int> host_devices() {
  const uint64_t m = g_host_mask.load(std::memory_order_acquire);
  std::vector<int> d;
  for (int i = 0; i < 64; ++i)
    if ((m >> i) & 1u) d.push_back(i);
  if (d.empty()) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) cur = 0;
    d.push_back(cur);
  }
  return d;
}

// span(i) = {lo, hi} of block i ({UINT64_MAX, 0}: an empty block, part of the group, no bytes)
template <class Span>
std::vector<HostGroup> plan_groups(uint64_t n, uint32_t ndev, uint64_t chunk, const Span& span) {
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const std::pair<uint64_t, uint64_t> sp = span(i);
    if (sp.second > sp.first) total += sp.second - sp.first;
  }
  const uint64_t nd = std::max<uint64_t>(1, std::min<uint64_t>(ndev, total / kStripeMinBytes));
  std::vector<HostGroup> groups;
  HostGroup g{0, 0, UINT64_MAX, 0, 0};
  uint64_t acc = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (g.count && g.dev + 1 < nd && acc >= (g.dev + 1) * (total / nd)) {  // the next device's share
      groups.push_back(g);
      g = HostGroup{i, 0, UINT64_MAX, 0, g.dev + 1};
    }
    const std::pair<uint64_t, uint64_t> sp = span(i);
    if (sp.second > sp.first) {
      const uint64_t lo = std::min(g.lo, sp.first), hi = std::max(g.hi, sp.second);
      if (g.count && g.lo != UINT64_MAX && hi - lo > chunk) {
        groups.push_back(g);
        g = HostGroup{i, 0, sp.first, sp.second, g.dev};
      } else {
        g.lo = lo;
        g.hi = hi;
      }
      acc += sp.second - sp.first;
    }
    ++g.count;
  }
  groups.push_back(g);
  for (auto& x : groups)
    if (x.lo == UINT64_MAX) x.lo = x.hi = 0;
  return groups;
}

// Two-slot staging pipeline over copy_stream (H2D) and stream (kernel + D2H).  The destructor drains
// both streams, so an early error return never leaves a copy in flight from host memory that is
// about to be freed.
struct SlotPipe {
  HostCtx* st;
  explicit SlotPipe(HostCtx* s) : st(s) {}
  ~SlotPipe() {
    (void)hipStreamSynchronize(st->copy_stream);
    (void)hipStreamSynchronize(st->stream);
  }
  // before group k's copies: slot k & 1 must be drained (group k - 2 done)
  hipError_t begin_copies(size_t k) const {
    return k >= 2 ? hipStreamWaitEvent(st->copy_stream, st->drained[k & 1], 0) : hipSuccess;
  }
  // after group k's copies: the kernel stream waits for them
  hipError_t end_copies(size_t k) const {
    hipError_t e = hipEventRecord(st->staged[k & 1], st->copy_stream);
    return e != hipSuccess ? e : hipStreamWaitEvent(st->stream, st->staged[k & 1], 0);
  }
  // after group k's kernel and result copies: slot k & 1 is free again
  hipError_t end_group(size_t k) const { return hipEventRecord(st->drained[k & 1], st->stream); }
};

// One device's share of a host batch: a locked host context of that device, its contiguous run of
// plan groups (blocks [first, first + count)) and their staging pipe.  (Members destroyed in reverse:
// the pipe drains its streams before the context is unlocked.)
struct HostLane {
  int device = -1;
  DevState* dev = nullptr;
  std::unique_ptr<CtxLock> cl;
  HostCtx* c = nullptr;
  std::vector<size_t> gi;
  uint64_t first = 0, count = 0;
  std::unique_ptr<SlotPipe> pipe;
};

struct DeviceRestore {  // the caller's current device, put back on every return
  int d = -1;
  DeviceRestore() { (void)hipGetDevice(&d); }
  ~DeviceRestore() {
    if (d >= 0) (void)hipSetDevice(d);
  }
};

// A host context on every device the plan uses, locked in ascending device order (two multi-device
// batches never wait on each other in a cycle).
int open_lanes(const std::vector<HostGroup>& groups, const std::vector<int>& devs, std::vector<HostLane>& lanes) {
  int nvis = 0;
  if (hipGetDeviceCount(&nvis) != hipSuccess || nvis <= 0)
    return fail(PDB_ENODEV, "no HIP device visible (pdb_crc32c has no CPU fallback)");
  lanes.clear();
  lanes.resize(devs.size());
  for (size_t k = 0; k < groups.size(); ++k) lanes[groups[k].dev].gi.push_back(k);
  for (size_t d = 0; d < devs.size(); ++d) {
    HostLane& L = lanes[d];
    if (L.gi.empty()) continue;
    L.device = devs[d];
    hipError_t e = hipSetDevice(L.device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    int rc = get_state(&L.dev);
    if (rc) return rc;
    L.cl.reset(new CtxLock(L.dev));
    L.c = L.cl->c;
    L.first = groups[L.gi.front()].first;
    for (size_t k : L.gi) L.count += groups[k].count;
  }
  return PDB_OK;
}

// Issue every lane's groups round-robin (group j of each device, then j + 1, ...), so all devices'
// copies start at once; issue(L, j) runs with L's device current.
template <class Issue>
int issue_lanes(std::vector<HostLane>& lanes, const Issue& issue) {
  for (size_t j = 0;; ++j) {
    bool any = false;
    for (HostLane& L : lanes) {
      if (j >= L.gi.size()) continue;
      any = true;
      hipError_t e = hipSetDevice(L.device);
      if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
      int rc = issue(L, j);
      if (rc) return rc;
    }
    if (!any) return PDB_OK;
  }
}

// Host batch over descriptors: per group, stage [lo, hi) of the host span, the rebased
// descriptors (and expected CRCs) in the workspace; H2D span + descriptors, kernel, D2H results.
int host_desc(const uint8_t* base, uint64_t base_len, const pdb_blk* blk, uint64_t nblk,
              uint32_t flags, int mode, const uint32_t* expected, uint32_t* out, uint8_t* ok,
              uint64_t* nbad_out) {
  if (nblk == 0) {
    if (nbad_out) *nbad_out = 0;
    return PDB_OK;
  }
  if (!base || !blk) return fail(PDB_EINVAL, "null argument");
  uint64_t n1k = 0, n4k = 0, n256 = 0, n512 = 0, n1023 = 0;  // size classes of the sized kernels
  uint32_t max_len = 0;
  for (uint64_t i = 0; i < nblk; ++i) {
    if (blk[i].off > base_len || blk[i].len > base_len - blk[i].off)
      return fail(PDB_ERANGE, "block " + std::to_string(i) + " exceeds base_len");
    max_len = std::max(max_len, blk[i].len);
    n1k += blk[i].len - 1024u <= 128u;
    n4k += blk[i].len - 4096u <= 256u;
    n256 += blk[i].len - 1u <= 255u;
    n512 += blk[i].len - 257u <= 255u;
    n1023 += blk[i].len - 513u <= 510u;
  }
  const std::vector<int> devs = host_devices();
  const std::vector<HostGroup> groups = plan_groups(nblk, static_cast<uint32_t>(devs.size()), host_chunk_bytes(), [&](uint64_t i) {
    return blk[i].len ? std::make_pair(blk[i].off & ~static_cast<uint64_t>(15), blk[i].off + blk[i].len)
                      : std::make_pair(UINT64_MAX, uint64_t{0});
  });
  // host-visible lengths pick the kernel: mostly WAL-record or sstable-block sized -> the sized
  // kernels (same results; the hint only changes speed)
  if (!(flags & (PDB_CRC_USE_INIT | PDB_CRC_SIZE_1K | PDB_CRC_SIZE_4K | PDB_CRC_SIZE_256 | PDB_CRC_SIZE_512 | PDB_CRC_SIZE_1023))) {
    if (4 * n1k >= 3 * nblk) flags |= PDB_CRC_SIZE_1K;
    else if (4 * n4k >= 3 * nblk) flags |= PDB_CRC_SIZE_4K;
    else if (4 * n256 >= 3 * nblk) flags |= small_records_prefer_512(blk, nblk) ? PDB_CRC_SIZE_512 : PDB_CRC_SIZE_256;
    else if (4 * (n256 + n512) >= 3 * nblk) flags |= PDB_CRC_SIZE_512;  // the 17-group window takes 1..512 B
    else if (4 * (n256 + n512 + n1023) >= 3 * nblk) flags |= PDB_CRC_SIZE_1023;  // 33 groups: 1..1024 B
    if ((flags & (PDB_CRC_SIZE_512 | PDB_CRC_SIZE_1023)) && mixed_lengths(blk, nblk, (flags & PDB_CRC_SIZE_512) ? 512u : 1023u))
      flags |= PDB_CRC_SIZE_MIXED;
  }
  DeviceRestore restore;
  std::vector<HostLane> lanes;
  int rc = open_lanes(groups, devs, lanes);
  if (rc) return rc;
  struct Geo {
    size_t off_desc = 0, off_out = 0, off_exp = 0, off_ok = 0, slot_bytes = 0, nslots = 1;
    uint32_t* d_nbad = nullptr;
    LongLane ll{};
    uint32_t nb = 0;
  };
  std::vector<Geo> geo(lanes.size());
  hipError_t e;
  for (size_t d = 0; d < lanes.size(); ++d) {
    HostLane& L = lanes[d];
    if (L.gi.empty()) continue;
    Geo& G = geo[d];
    if ((e = hipSetDevice(L.device)) != hipSuccess) return hip_fail(e, "hipSetDevice");
    size_t need = 0;
    uint64_t max_count = 0;
    for (size_t k : L.gi) {
      need = std::max<size_t>(need, groups[k].hi - groups[k].lo);
      max_count = std::max(max_count, groups[k].count);
    }
    G.off_desc = align_up(need + 16, 256);
    G.off_out = align_up(G.off_desc + max_count * sizeof(pdb_blk), 256);
    G.off_exp = align_up(G.off_out + max_count * sizeof(uint32_t), 256);
    G.off_ok = align_up(G.off_exp + (mode == kModeVerify ? max_count * 4 : 0), 256);
    G.slot_bytes = align_up(G.off_ok + (mode == kModeVerify ? max_count : 0), 256);
    G.nslots = L.gi.size() > 1 ? 2 : 1;
    if ((rc = ensure_ws(L.c, G.nslots * G.slot_bytes + 256))) return rc;
    // blocks of >= 16 KiB: the long-block lane on this context's stream (crc32c_internal.h)
    if (max_len >= kLongMinBytes && !L.c->d_lane && (rc = alloc_lane(L.c->stream, &L.c->d_lane))) return rc;
    G.ll = long_lane_at(max_len >= kLongMinBytes ? L.c->d_lane : nullptr, L.dev->d_pow2);
    G.d_nbad = reinterpret_cast<uint32_t*>(L.c->d_ws + G.nslots * G.slot_bytes);
    L.pipe.reset(new SlotPipe(L.c));
    if (mode == kModeVerify && (e = hipMemsetAsync(G.d_nbad, 0, 4, L.c->stream)) != hipSuccess)
      return hip_fail(e, "hipMemsetAsync");
  }
  std::vector<std::vector<pdb_blk>> rbs(groups.size());  // async H2D sources, alive until the drain
  rc = issue_lanes(lanes, [&](HostLane& L, size_t k) -> int {
    const Geo& G = geo[&L - lanes.data()];
    const HostGroup& x = groups[L.gi[k]];
    HostCtx* st = L.c;
    hipStream_t s = st->stream, cs = st->copy_stream;
    uint8_t* ws = st->d_ws + (k % G.nslots) * G.slot_bytes;
    std::vector<pdb_blk>& rb = rbs[L.gi[k]];
    rb.assign(blk + x.first, blk + x.first + x.count);
    for (auto& b : rb) b.off = b.len ? b.off - x.lo : 0;
    hipError_t e2;
    if ((e2 = L.pipe->begin_copies(k)) != hipSuccess) return hip_fail(e2, "hipStreamWaitEvent");
    if (x.hi > x.lo && (e2 = hipMemcpyAsync(ws, base + x.lo, x.hi - x.lo, hipMemcpyHostToDevice, cs)) != hipSuccess)
      return hip_fail(e2, "hipMemcpyAsync(span)");
    if ((e2 = hipMemcpyAsync(ws + G.off_desc, rb.data(), x.count * sizeof(pdb_blk), hipMemcpyHostToDevice, cs)) != hipSuccess)
      return hip_fail(e2, "hipMemcpyAsync(desc)");
    if (mode == kModeVerify &&
        (e2 = hipMemcpyAsync(ws + G.off_exp, expected + x.first, x.count * 4, hipMemcpyHostToDevice, cs)) != hipSuccess)
      return hip_fail(e2, "hipMemcpyAsync(expected)");
    if ((e2 = L.pipe->end_copies(k)) != hipSuccess) return hip_fail(e2, "hipEventRecord(staged)");
    e2 = launch_desc(L.dev->hgeom, L.dev->d_tables, ws, reinterpret_cast<const pdb_blk*>(ws + G.off_desc), x.count, flags,
                     mode, reinterpret_cast<const uint32_t*>(ws + G.off_exp), reinterpret_cast<uint32_t*>(ws + G.off_out),
                     ws + G.off_ok, G.d_nbad, s, G.ll.hdr ? &G.ll : nullptr);
    if (e2 != hipSuccess) return hip_fail(e2, "launch_desc");
    if (mode == kModeOut) {
      if ((e2 = hipMemcpyAsync(out + x.first, ws + G.off_out, x.count * 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return hip_fail(e2, "hipMemcpyAsync(out)");
    } else if (ok && (e2 = hipMemcpyAsync(ok + x.first, ws + G.off_ok, x.count, hipMemcpyDeviceToHost, s)) != hipSuccess) {
      return hip_fail(e2, "hipMemcpyAsync(ok)");
    }
    if ((e2 = L.pipe->end_group(k)) != hipSuccess) return hip_fail(e2, "hipEventRecord(drained)");
    return PDB_OK;
  });
  if (rc) return rc;
  uint64_t nb = 0;
  for (size_t d = 0; d < lanes.size(); ++d) {
    HostLane& L = lanes[d];
    if (L.gi.empty()) continue;
    if ((e = hipSetDevice(L.device)) != hipSuccess) return hip_fail(e, "hipSetDevice");
    if (mode == kModeVerify && (e = hipMemcpyAsync(&geo[d].nb, geo[d].d_nbad, 4, hipMemcpyDeviceToHost, L.c->stream)) != hipSuccess)
      return hip_fail(e, "hipMemcpyAsync(nbad)");
  }
  for (size_t d = 0; d < lanes.size(); ++d) {
    if (lanes[d].gi.empty()) continue;
    if ((e = hipStreamSynchronize(lanes[d].c->stream)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    nb += geo[d].nb;
  }
  if (nbad_out) *nbad_out = nb;
  return PDB_OK;
}

constexpr uint64_t kSpanMaxBytes = 1ull << 45;        // 16383 segments of <= 2 GiB
constexpr uint64_t kSpanHostThreshold = 8ull << 20;  // scalar Extend: device-copy spans >= 8 MiB
constexpr uint64_t kScalarOneLeaf = 64ull << 10;     // below: one launch, one wave; above: span split

// Scalar Extend below kSpanHostThreshold (the per-record / per-block call of log_writer.cc:121,
// table_builder.cc:197-199, format.cc:97): latency-bound, so no DMA copies at all -- the bytes are
// staged in pinned mapped memory, read by the kernel across PCIe, and the CRC is written back into
// the same mapping.  < 64 KiB: one launch_fixed of one block; larger: launch_span (parallel 64-KiB
// segments + tree combine, scratch in the device workspace).
int host_scalar(uint32_t init, const uint8_t* data, uint64_t n, uint32_t* out) {
  DevState* st;
  int rc = get_state(&st);
  if (rc) return rc;
  if (st->scalar_mode == kScalarServer && n <= kServerCap) return server_call(st, init, data, n, out);
  // launch per call (> 64 KiB, or the A/B modes): the pinned stage (st->mu) and a host context
  std::lock_guard<std::mutex> lk(st->mu);
  CtxLock cl(st);
  hipError_t e = hipSetDevice(st->device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  if ((rc = ensure_stage(st, kStageHdr + align_up(n, 256)))) return rc;
  memcpy(st->h_stage + kStageHdr, data, n);
  uint32_t* d_res = reinterpret_cast<uint32_t*>(st->d_stage);
  volatile uint32_t* h_res = reinterpret_cast<volatile uint32_t*>(st->h_stage);
  hipStream_t s = cl.c->stream;
  if (n < kScalarOneLeaf) {
    // The kernel's only host write is the result, after its last read of the staged bytes, so
    // seeing it change means the call is complete: spin on it instead of waiting for the
    // end-of-kernel signal.  A CRC equal to the sentinel just falls through to the stream sync.
    const uint32_t sentinel = st->seq++ * 0x9E3779B9u ^ 0x5A5A5A5Au;
    *h_res = sentinel;
    LaunchGeom hgeom = st->hgeom;
    e = launch_fixed(hgeom, st->d_tables, st->d_stage + kStageHdr, 0, static_cast<uint32_t>(n), 1,
                     PDB_CRC_USE_INIT, init, d_res, s);
    if (e != hipSuccess) return hip_fail(e, "launch_fixed(scalar)");
    if (st->scalar_mode == kScalarPoll) {
      if (!st->stage_done && (e = hipEventCreateWithFlags(&st->stage_done, hipEventDisableTiming)) != hipSuccess)
        return hip_fail(e, "hipEventCreate(stage)");
      if ((e = hipEventRecord(st->stage_done, s)) != hipSuccess) return hip_fail(e, "hipEventRecord(stage)");
      st->stage_pending = true;
      for (uint32_t spin = 0; spin < (1u << 22); ++spin) {
        const uint32_t v = *h_res;
        if (v != sentinel) {
          *out = v;
          return PDB_OK;
        }
        __builtin_ia32_pause();
      }
    }
  } else {
    if ((rc = ensure_ws(cl.c, span_scratch_words(n) * 4 + 256))) return rc;
    e = launch_span(st->hgeom, st->d_tables, st->d_pow2, init, st->d_stage + kStageHdr, n,
                    reinterpret_cast<uint32_t*>(cl.c->d_ws), d_res, s);
    if (e != hipSuccess) return hip_fail(e, "launch_span(scalar)");
  }
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  *out = *h_res;
  return PDB_OK;
}

// Scalar Extend over a long host span: H2D, parallel segments + tree combine, 4-byte D2H.
int host_span(uint32_t init, const uint8_t* data, uint64_t n, uint32_t* out) {
  if (n > kSpanMaxBytes) return fail(PDB_ERANGE, "span longer than 2^45 bytes");
  DevState* dev;
  int rc = get_state(&dev);
  if (rc) return rc;
  CtxLock cl(dev);
  HostCtx* st = cl.c;
  hipError_t e = hipSetDevice(dev->device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  const size_t off_scr = align_up(n + 16, 256);
  const size_t off_out = align_up(off_scr + span_scratch_words(n) * 4, 256);
  rc = ensure_ws(st, off_out + 256);
  if (rc) return rc;
  hipStream_t s = st->stream;
  uint8_t* ws = st->d_ws;
  if ((e = hipMemcpyAsync(ws, data, n, hipMemcpyHostToDevice, s)) != hipSuccess)
    return hip_fail(e, "hipMemcpyAsync(span)");
  e = launch_span(dev->hgeom, dev->d_tables, dev->d_pow2, init, ws, n, reinterpret_cast<uint32_t*>(ws + off_scr),
                  reinterpret_cast<uint32_t*>(ws + off_out), s);
  if (e != hipSuccess) return hip_fail(e, "launch_span");
  if ((e = hipMemcpyAsync(out, ws + off_out, 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
    return hip_fail(e, "hipMemcpyAsync(out)");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  return PDB_OK;
}

// host_sst on a buffer from pdb_host_alloc (d_buf: its device mapping): no DMA at all -- the sst
// kernel reads the blocks across PCIe through the mapping and a seal writes the trailers in place
// the same way (the device seal's own kernel, crc_sst4k_kernel<SstSrc, ParkSealSink>), the handles
// and the verify's ok bytes in the context's pinned scratch; one launch and one synchronisation
// (tools/seal_batches.py: 4-MiB batches 31 -> 40.5 GiB/s, 16 MiB 43 -> 46, the bare H2D copy 44 / 51).
// Blocks longer than kLongBlock (a table's index and filter blocks: 16 KiB .. 1.3 MiB in the engine)
// are left out of that kernel, whose slow path hashes a block on one wave -- a round trip across
// PCIe per 16 KiB, 0.3-1.3 ms for the last batch of a large table (profiles/r05/engine/long_blocks/)
// -- and hashed in 4-KiB pieces on as many waves instead: one descriptor launch over all of the
// batch's long blocks and one combine launch (launch_span_many), on the same stream; the host writes
// their trailers (seal) or checks them (verify) after the synchronisation.
constexpr uint64_t kLongBlock = 16u << 10;
// PDB_LONG_BLOCK=<bytes> (read once; 0: never) moves the threshold, for A/B runs
uint64_t long_block_bytes() {
  static const uint64_t v = [] {
    const char* e = getenv("PDB_LONG_BLOCK");
    if (!e) return kLongBlock;
    const unsigned long long x = strtoull(e, nullptr, 10);
    return x ? static_cast<uint64_t>(x) : UINT64_MAX;
  }();
  return v;
}
int host_sst_mapped(uint8_t* h_buf, uint8_t* d_buf, uint64_t buf_len, const pdb_block_handle* h, uint64_t n, bool seal,
                    uint8_t* ok, int64_t* nbad_out) {
  const bool stamp = seal_stamps_on();
  SealStamp ss{buf_len, stamp ? mono_ns() : 0, 0, 0, 0, g_pin_allocs.load(std::memory_order_relaxed), n, 0, 0.f};
  if (stamp)
    for (uint64_t i = 0; i < n; ++i) ss.maxblk = std::max<uint64_t>(ss.maxblk, h[i].size);
  // the long blocks (their handle indices) and the scratch their span launches share
  // Long blocks of up to 2^14 pieces of 4 KiB (64 MiB) go together: one descriptor launch over all
  // their pieces, one combine launch; longer ones each take launch_span (its scratch).
  constexpr uint64_t kPiece = 4096, kMaxPieces = 1ull << PDB_SPAN_MAX_SEGS_LOG2;
  std::vector<uint64_t> longs;
  uint64_t scratch_words = 0, npieces = 0, nmany = 0;
  const uint64_t long_block = long_block_bytes();
  for (uint64_t i = 0; i < n; ++i)
    if (h[i].size >= long_block) {
      longs.push_back(i);
      const uint64_t pieces = (h[i].size + 1 + kPiece - 1) / kPiece;
      if (pieces <= kMaxPieces) {
        npieces += pieces;
        ++nmany;
      } else {
        scratch_words = std::max<uint64_t>(scratch_words, span_scratch_words(h[i].size + 1, 12));
      }
    }
  const uint64_t nl = longs.size(), m = n - nl;  // m: blocks the sst kernel takes
  DevState* dev;
  int rc = get_state(&dev);
  if (rc) return rc;
  CtxLock cl(dev);
  HostCtx* st = cl.c;
  struct StampEvents {  // (destroyed on every return)
    hipEvent_t e[2] = {nullptr, nullptr};
    ~StampEvents() {
      for (hipEvent_t x : e)
        if (x) (void)hipEventDestroy(x);
    }
  } sev;
  hipEvent_t* ev = sev.e;
  if (stamp) {
    ss.t1 = mono_ns();
    if (hipEventCreate(&ev[0]) != hipSuccess || hipEventCreate(&ev[1]) != hipSuccess) return fail(PDB_EHIP, "hipEventCreate(stamps)");
  }
  hipError_t e = hipSetDevice(dev->device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  // pinned: [the kernel's handles][ok bytes, 128-B lines][nbad][the long blocks' CRCs][their pieces][their parts]
  const size_t pin_ok = align_up(n * sizeof(pdb_block_handle), 128);  // (the verify stores 128-B lines of ok bytes)
  const size_t pin_nb = pin_ok + align_up(n, 64), pin_long = pin_nb + 64;
  const size_t pin_pieces = pin_long + align_up(4 * nl, 64), pin_parts = pin_pieces + npieces * sizeof(pdb_blk);
  if ((rc = ensure_pin(st, pin_parts + nmany * sizeof(SpanPart)))) return rc;
  if (!st->d_pin) return fail(PDB_EHIP, "pinned scratch has no device mapping");
  // device workspace: [nbad][span scratch][the pieces' leaves] (the long blocks' CRCs: pinned)
  const size_t ws_scr = 256;
  const size_t ws_leaves = ws_scr + align_up(scratch_words * 4, 256);
  if ((rc = ensure_ws(st, ws_leaves + npieces * 4 + 256))) return rc;
  pdb_block_handle* hk = reinterpret_cast<pdb_block_handle*>(st->h_pin);
  if (nl == 0) {
    memcpy(hk, h, n * sizeof(pdb_block_handle));
  } else {
    for (uint64_t i = 0, j = 0; i < n; ++i)
      if (h[i].size < long_block) hk[j++] = h[i];
  }
  hipStream_t s = st->stream;
  uint32_t* d_nbad = reinterpret_cast<uint32_t*>(st->d_ws);
  uint32_t* d_long = reinterpret_cast<uint32_t*>(st->d_pin + pin_long);  // (written across PCIe: no copy back)
  uint32_t* d_scr = reinterpret_cast<uint32_t*>(st->d_ws + ws_scr);
  uint32_t* h_nb = reinterpret_cast<uint32_t*>(st->h_pin + pin_nb);
  uint32_t* h_long = reinterpret_cast<uint32_t*>(st->h_pin + pin_long);
  *h_nb = 0;
  if (!seal && (e = hipMemsetAsync(d_nbad, 0, 4, s)) != hipSuccess) return hip_fail(e, "hipMemsetAsync");
  if (stamp) (void)hipEventRecord(ev[0], s);
  e = launch_sst(dev->hgeom, dev->d_tables, d_buf, buf_len, reinterpret_cast<const pdb_block_handle*>(st->d_pin), m, seal,
                 seal ? nullptr : st->d_pin + pin_ok, seal ? nullptr : d_nbad, s);
  if (e != hipSuccess) return hip_fail(e, seal ? "launch_sst(seal, mapped)" : "launch_sst(verify, mapped)");
  // Value(contents || type) of each long block: the ones of <= 2^14 pieces first (their CRCs at
  // d_long[0, nmany)), then the rest (d_long[nmany, nl)); `order` maps back to longs[]
  std::vector<uint64_t> order;
  order.reserve(nl);
  if (nmany) {
    pdb_blk* pc = reinterpret_cast<pdb_blk*>(st->h_pin + pin_pieces);
    SpanPart* parts = reinterpret_cast<SpanPart*>(st->h_pin + pin_parts);
    uint64_t q = 0, b = 0;
    for (uint64_t k = 0; k < nl; ++k) {
      const pdb_block_handle& hb = h[longs[k]];
      const uint64_t L = hb.size + 1, pieces = (L + kPiece - 1) / kPiece;
      if (pieces > kMaxPieces) continue;
      // the first piece takes the Value seed and the bytes that are not a whole piece
      const uint64_t first = L - (pieces - 1) * kPiece;
      uint32_t ml = 0;
      while ((1ull << ml) < pieces) ++ml;
      parts[b++] = SpanPart{static_cast<uint32_t>(q), static_cast<uint32_t>(pieces), ml, 0u};
      pc[q++] = pdb_blk{hb.offset, static_cast<uint32_t>(first), 0u};
      for (uint64_t j = 1; j < pieces; ++j)
        pc[q++] = pdb_blk{hb.offset + first + (j - 1) * kPiece, static_cast<uint32_t>(kPiece), 0xFFFFFFFFu};
      order.push_back(k);
    }
    e = launch_span_many(dev->hgeom, dev->d_tables, dev->d_pow2, d_buf, reinterpret_cast<const pdb_blk*>(st->d_pin + pin_pieces),
                         npieces, reinterpret_cast<const SpanPart*>(st->d_pin + pin_parts), static_cast<uint32_t>(nmany), 12,
                         reinterpret_cast<uint32_t*>(st->d_ws + ws_leaves), d_long, s);
    if (e != hipSuccess) return hip_fail(e, "launch_span_many(long blocks, mapped)");
  }
  for (uint64_t k = 0; k < nl; ++k) {
    const pdb_block_handle& b = h[longs[k]];
    if ((b.size + 1 + kPiece - 1) / kPiece <= kMaxPieces) continue;
    e = launch_span(dev->hgeom, dev->d_tables, dev->d_pow2, 0u, d_buf + b.offset, b.size + 1, d_scr,
                    d_long + order.size(), s, 12);
    if (e != hipSuccess) return hip_fail(e, "launch_span(long block, mapped)");
    order.push_back(k);
  }
  // h_long[r] is the CRC of longs[order[r]]: crc_of[k] for longs[k]
  std::vector<uint32_t> crc_of(nl);
  if (stamp) {
    (void)hipEventRecord(ev[1], s);
    ss.t2 = mono_ns();
  }
  if (!seal && (e = hipMemcpyAsync(h_nb, d_nbad, 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
    return hip_fail(e, "hipMemcpyAsync(nbad)");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  if (stamp) {
    ss.t3 = mono_ns();
    (void)hipEventElapsedTime(&ss.kern_ms, ev[0], ev[1]);
    std::lock_guard<std::mutex> lk(g_seal_stamp_mu);
    g_seal_stamps.push_back(ss);
  }
  for (uint64_t r = 0; r < nl; ++r) crc_of[order[r]] = h_long[r];
  // the long blocks' trailers: [type][Mask(crc)] little-endian at offset + size (table_builder.cc:197-200)
  uint64_t nbad = seal ? 0 : *h_nb;
  const uint8_t* okk = st->h_pin + pin_ok;  // the kernel's ok bytes, in the order of its handles
  for (uint64_t k = 0; k < nl; ++k) {
    const pdb_block_handle& b = h[longs[k]];
    uint8_t* tr = h_buf + b.offset + b.size + 1;
    if (seal) {
      const uint32_t w = pdb_mask(crc_of[k]);
      tr[0] = static_cast<uint8_t>(w);
      tr[1] = static_cast<uint8_t>(w >> 8);
      tr[2] = static_cast<uint8_t>(w >> 16);
      tr[3] = static_cast<uint8_t>(w >> 24);
    } else {
      const uint32_t w = static_cast<uint32_t>(tr[0]) | (static_cast<uint32_t>(tr[1]) << 8) |
                         (static_cast<uint32_t>(tr[2]) << 16) | (static_cast<uint32_t>(tr[3]) << 24);
      nbad += pdb_unmask(w) != crc_of[k];
    }
  }
  if (!seal && ok) {
    if (nl == 0) {
      memcpy(ok, okk, n);
    } else {
      for (uint64_t i = 0, j = 0, k = 0; i < n; ++i) {
        if (k < nl && longs[k] == i) {
          const pdb_block_handle& b = h[i];
          const uint8_t* tr = h_buf + b.offset + b.size + 1;
          const uint32_t w = static_cast<uint32_t>(tr[0]) | (static_cast<uint32_t>(tr[1]) << 8) |
                             (static_cast<uint32_t>(tr[2]) << 16) | (static_cast<uint32_t>(tr[3]) << 24);
          ok[i] = pdb_unmask(w) == crc_of[k] ? 1u : 0u;
          ++k;
        } else {
          ok[i] = okk[j++];
        }
      }
    }
  }
  if (nbad_out) *nbad_out = static_cast<int64_t>(nbad);
  return PDB_OK;
}

int host_sst(uint8_t* buf, uint64_t buf_len, const pdb_block_handle* h, uint64_t n, bool seal,
             uint8_t* ok, int64_t* nbad_out) {
  if (n == 0) {
    if (nbad_out) *nbad_out = 0;
    return PDB_OK;
  }
  if (!buf || !h) return fail(PDB_EINVAL, "null argument");
  for (uint64_t i = 0; i < n; ++i) {
    // block + 5-byte trailer must lie inside the buffer (table/format.cc:84-87 "truncated")
    if (h[i].offset > buf_len || h[i].size > buf_len - h[i].offset ||
        buf_len - h[i].offset - h[i].size < 5)
      return fail(PDB_ERANGE, "block handle " + std::to_string(i) + " (+trailer) exceeds buffer");
    if (h[i].size + 1 > 0xFFFFFFFFull) return fail(PDB_ERANGE, "block larger than 4 GiB");
  }
  // PDB_HOST_MAPPED=0 (read once per process): pinned buffers take the DMA route below as well
  // (experiments: the engine's seals by DMA against zero-copy, profiles/r05/engine/)
  static const bool mapped = [] {
    const char* e = getenv("PDB_HOST_MAPPED");
    return !(e && e[0] == '0');
  }();
  if (mapped)
    if (uint8_t* d_buf = pin_mapping(buf, buf_len)) return host_sst_mapped(buf, d_buf, buf_len, h, n, seal, ok, nbad_out);
  // staging groups of at most host_chunk_bytes() of span (block + trailer), striped over the devices
  const std::vector<int> devs = host_devices();
  const std::vector<HostGroup> groups = plan_groups(n, static_cast<uint32_t>(devs.size()), host_chunk_bytes(), [&](uint64_t i) {
    return std::make_pair(h[i].offset & ~static_cast<uint64_t>(15), h[i].offset + h[i].size + 5);
  });
  // Long blocks (as in host_sst_mapped, up to 2^14 pieces of 4 KiB): the sst kernel gets a 0-byte
  // stand-in at the block's offset (its type byte alone: cheap, and nothing it writes lands in the
  // image) and launch_span_many hashes the block from the group's staged copy; the host then puts
  // the block's masked CRC (seal) or its check (verify, correcting the stand-in's verdict) in place
  // (one 400-KiB block in a 16-MiB batch: +210 us on this route before, profiles/r05/engine/long_blocks/).
  constexpr uint64_t kPiece = 4096, kMaxPieces = 1ull << PDB_SPAN_MAX_SEGS_LOG2;
  const uint64_t long_block = long_block_bytes();
  auto is_long = [&](const pdb_block_handle& b) {
    return b.size >= long_block && (b.size + 1 + kPiece - 1) / kPiece <= kMaxPieces;
  };
  DeviceRestore restore;
  std::vector<HostLane> lanes;
  int rc = open_lanes(groups, devs, lanes);
  if (rc) return rc;
  // per lane: its slots; its pinned scratch holds, for ITS blocks (index - first): the rebased handles,
  // the trailer words (seal) or ok bytes (verify), nbad, then its long blocks' CRCs, pieces and parts
  struct Geo {
    size_t off_h = 0, off_ok = 0, slot_bytes = 0, nslots = 1, ws_leaves = 0;
    size_t pin_crc = 0, pin_lcrc = 0, pin_pieces = 0, pin_parts = 0;
    std::vector<uint64_t> longs;  // its long blocks (handle indices, ascending)
    uint64_t lq = 0, lp = 0;      // the next long block / piece (across its groups)
    uint32_t* d_nbad = nullptr;
  };
  std::vector<Geo> geo(lanes.size());
  hipError_t e;
  for (size_t d = 0; d < lanes.size(); ++d) {
    HostLane& L = lanes[d];
    if (L.gi.empty()) continue;
    Geo& G = geo[d];
    if ((e = hipSetDevice(L.device)) != hipSuccess) return hip_fail(e, "hipSetDevice");
    size_t need = 0;
    uint64_t max_count = 0, npieces = 0, max_gpieces = 0;
    for (size_t k : L.gi) {
      const HostGroup& x = groups[k];
      need = std::max<size_t>(need, x.hi - x.lo);
      max_count = std::max(max_count, x.count);
      uint64_t gp = 0;
      for (uint64_t i = x.first; i < x.first + x.count; ++i)
        if (is_long(h[i])) {
          G.longs.push_back(i);
          gp += (h[i].size + 1 + kPiece - 1) / kPiece;
        }
      npieces += gp;
      max_gpieces = std::max(max_gpieces, gp);
    }
    G.off_h = align_up(need + 16, 256);
    G.off_ok = align_up(G.off_h + max_count * sizeof(pdb_block_handle), 256);
    G.slot_bytes = align_up(G.off_ok + 4 * max_count, 256);  // ok bytes (verify) or masked CRCs (seal)
    G.nslots = L.gi.size() > 1 ? 2 : 1;
    // device: the slots, nbad, then the long blocks' leaves (one group's at a time: stream s)
    G.ws_leaves = G.nslots * G.slot_bytes + 256;
    if ((rc = ensure_ws(L.c, G.ws_leaves + align_up(4 * max_gpieces, 256)))) return rc;
    const uint64_t nl = G.longs.size();
    G.pin_crc = align_up(L.count * sizeof(pdb_block_handle), 64);
    G.pin_lcrc = G.pin_crc + align_up(4 * L.count, 64) + 64;
    G.pin_pieces = G.pin_lcrc + align_up(4 * nl, 64);
    G.pin_parts = G.pin_pieces + npieces * sizeof(pdb_blk);
    if ((rc = ensure_pin(L.c, G.pin_parts + nl * sizeof(SpanPart)))) return rc;
    if (nl && !L.c->d_pin) return fail(PDB_EHIP, "pinned scratch has no device mapping");
    *reinterpret_cast<uint32_t*>(L.c->h_pin + G.pin_crc + align_up(4 * L.count, 64)) = 0;
    G.d_nbad = reinterpret_cast<uint32_t*>(L.c->d_ws + G.nslots * G.slot_bytes);
    L.pipe.reset(new SlotPipe(L.c));
    if (!seal && (e = hipMemsetAsync(G.d_nbad, 0, 4, L.c->stream)) != hipSuccess) return hip_fail(e, "hipMemsetAsync");
  }
  // Seal: only the 4 CRC bytes of every trailer change, so the kernel writes the masked CRCs into
  // a compact array, 4 B per block come back across PCIe (not the span), and the host encodes
  // them little-endian at offset + size + 1 (table_builder.cc:199-200).
  rc = issue_lanes(lanes, [&](HostLane& L, size_t k) -> int {
    Geo& G = geo[&L - lanes.data()];
    const HostGroup& x = groups[L.gi[k]];
    HostCtx* st = L.c;
    hipStream_t s = st->stream, cs = st->copy_stream;
    const LaunchGeom& hgeom = L.dev->hgeom;
    uint8_t* ws = st->d_ws + (k % G.nslots) * G.slot_bytes;
    const uint64_t li = x.first - L.first;  // the group's first block in the lane's arrays
    pdb_block_handle* rh = reinterpret_cast<pdb_block_handle*>(st->h_pin) + li;  // async H2D sources
    for (uint64_t i = 0; i < x.count; ++i)
      rh[i] = pdb_block_handle{h[x.first + i].offset - x.lo, is_long(h[x.first + i]) ? 0u : h[x.first + i].size};
    hipError_t e2;
    if ((e2 = L.pipe->begin_copies(k)) != hipSuccess) return hip_fail(e2, "hipStreamWaitEvent");
    if ((e2 = hipMemcpyAsync(ws, buf + x.lo, x.hi - x.lo, hipMemcpyHostToDevice, cs)) != hipSuccess)
      return hip_fail(e2, "hipMemcpyAsync(span)");
    if ((e2 = hipMemcpyAsync(ws + G.off_h, rh, x.count * sizeof(pdb_block_handle), hipMemcpyHostToDevice, cs)) != hipSuccess)
      return hip_fail(e2, "hipMemcpyAsync(handles)");
    if ((e2 = L.pipe->end_copies(k)) != hipSuccess) return hip_fail(e2, "hipEventRecord(staged)");
    const pdb_block_handle* d_h = reinterpret_cast<const pdb_block_handle*>(ws + G.off_h);
    uint8_t* pin_res = st->h_pin + G.pin_crc;
    if (seal) {
      uint32_t* d_crc = reinterpret_cast<uint32_t*>(ws + G.off_ok);
      if ((e2 = launch_sst_masked(hgeom, L.dev->d_tables, ws, x.hi - x.lo, d_h, x.count, d_crc, s)) != hipSuccess)
        return hip_fail(e2, "launch_sst_masked");
      if ((e2 = hipMemcpyAsync(reinterpret_cast<uint32_t*>(pin_res) + li, d_crc, x.count * 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return hip_fail(e2, "hipMemcpyAsync(crcs)");
    } else {
      if ((e2 = launch_sst(hgeom, L.dev->d_tables, ws, x.hi - x.lo, d_h, x.count, false, ws + G.off_ok, G.d_nbad, s)) !=
          hipSuccess)
        return hip_fail(e2, "launch_sst");
      if ((ok || !G.longs.empty()) &&
          (e2 = hipMemcpyAsync(pin_res + li, ws + G.off_ok, x.count, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return hip_fail(e2, "hipMemcpyAsync(ok)");
    }
    // the group's long blocks: their pieces (offsets in the staged copy) and parts, pinned and
    // mapped; CRCs to the lane's long-CRC words [lq0, lq)
    const uint64_t nl = G.longs.size(), lq0 = G.lq, lp0 = G.lp;
    pdb_blk* pc = reinterpret_cast<pdb_blk*>(st->h_pin + G.pin_pieces);
    SpanPart* parts = reinterpret_cast<SpanPart*>(st->h_pin + G.pin_parts);
    for (; G.lq < nl && G.longs[G.lq] < x.first + x.count; ++G.lq) {
      const pdb_block_handle& hb = h[G.longs[G.lq]];
      const uint64_t Lb = hb.size + 1, pieces = (Lb + kPiece - 1) / kPiece, first = Lb - (pieces - 1) * kPiece;
      uint32_t ml = 0;
      while ((1ull << ml) < pieces) ++ml;
      parts[G.lq] = SpanPart{static_cast<uint32_t>(G.lp - lp0), static_cast<uint32_t>(pieces), ml, 0u};
      const uint64_t o = hb.offset - x.lo;
      pc[G.lp++] = pdb_blk{o, static_cast<uint32_t>(first), 0u};
      for (uint64_t j = 1; j < pieces; ++j)
        pc[G.lp++] = pdb_blk{o + first + (j - 1) * kPiece, static_cast<uint32_t>(kPiece), 0xFFFFFFFFu};
    }
    if (G.lq > lq0) {
      uint32_t* d_lcrc = reinterpret_cast<uint32_t*>(st->d_pin + G.pin_lcrc) + lq0;  // (written across PCIe)
      e2 = launch_span_many(hgeom, L.dev->d_tables, L.dev->d_pow2, ws, reinterpret_cast<const pdb_blk*>(st->d_pin + G.pin_pieces) + lp0,
                            G.lp - lp0, reinterpret_cast<const SpanPart*>(st->d_pin + G.pin_parts) + lq0,
                            static_cast<uint32_t>(G.lq - lq0), 12, reinterpret_cast<uint32_t*>(st->d_ws + G.ws_leaves), d_lcrc, s);
      if (e2 != hipSuccess) return hip_fail(e2, "launch_span_many(long blocks)");
    }
    if ((e2 = L.pipe->end_group(k)) != hipSuccess) return hip_fail(e2, "hipEventRecord(drained)");
    return PDB_OK;
  });
  if (rc) return rc;
  for (size_t d = 0; d < lanes.size(); ++d) {
    HostLane& L = lanes[d];
    if (L.gi.empty() || seal) continue;
    if ((e = hipSetDevice(L.device)) != hipSuccess) return hip_fail(e, "hipSetDevice");
    uint32_t* h_nb = reinterpret_cast<uint32_t*>(L.c->h_pin + geo[d].pin_crc + align_up(4 * L.count, 64));
    if ((e = hipMemcpyAsync(h_nb, geo[d].d_nbad, 4, hipMemcpyDeviceToHost, L.c->stream)) != hipSuccess)
      return hip_fail(e, "hipMemcpyAsync(nbad)");
  }
  for (HostLane& L : lanes)
    if (!L.gi.empty() && (e = hipStreamSynchronize(L.c->stream)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  int64_t nbad = 0;
  for (size_t d = 0; d < lanes.size(); ++d) {
    HostLane& L = lanes[d];
    if (L.gi.empty()) continue;
    const Geo& G = geo[d];
    uint32_t* crc = reinterpret_cast<uint32_t*>(L.c->h_pin + G.pin_crc);  // (seal) lane-local
    uint8_t* h_ok = L.c->h_pin + G.pin_crc;                                  // (verify) lane-local
    const uint32_t* h_lcrc = reinterpret_cast<const uint32_t*>(L.c->h_pin + G.pin_lcrc);
    if (!seal) nbad += *reinterpret_cast<const uint32_t*>(L.c->h_pin + G.pin_crc + align_up(4 * L.count, 64));
    for (uint64_t q = 0; q < G.longs.size(); ++q) {  // the long blocks in place of their stand-ins
      const uint64_t i = G.longs[q], li = i - L.first;
      if (seal) {
        crc[li] = pdb_mask(h_lcrc[q]);
      } else {
        const uint8_t* tr = buf + h[i].offset + h[i].size + 1;
        const uint32_t w = static_cast<uint32_t>(tr[0]) | (static_cast<uint32_t>(tr[1]) << 8) |
                           (static_cast<uint32_t>(tr[2]) << 16) | (static_cast<uint32_t>(tr[3]) << 24);
        const uint8_t good = pdb_unmask(w) == h_lcrc[q] ? 1u : 0u;
        nbad += (h_ok[li] ? 0 : -1) + (good ? 0 : 1);
        h_ok[li] = good;
      }
    }
    if (seal) {
      for (uint64_t li = 0; li < L.count; ++li) {
        const pdb_block_handle& b = h[L.first + li];
        uint8_t* tr = buf + b.offset + b.size + 1;
        tr[0] = static_cast<uint8_t>(crc[li]);
        tr[1] = static_cast<uint8_t>(crc[li] >> 8);
        tr[2] = static_cast<uint8_t>(crc[li] >> 16);
        tr[3] = static_cast<uint8_t>(crc[li] >> 24);
      }
    } else if (ok) {
      memcpy(ok + L.first, h_ok, L.count);
    }
  }
  if (nbad_out) *nbad_out = nbad;
  return PDB_OK;
}

// The striping plan of a host descriptor batch over `ndev` devices, for tests (pdb_host_stripe_plan)
int64_t stripe_plan(const pdb_blk* blk, uint64_t nblk, uint32_t ndev, uint64_t chunk, uint64_t* first, uint32_t* dev,
                    uint64_t cap) {
  if (!ndev || ndev > 64) return fail(PDB_EINVAL, "ndev must be 1..64");
  const std::vector<HostGroup> g = plan_groups(nblk, ndev, chunk ? chunk : host_chunk_bytes(), [&](uint64_t i) {
    return blk[i].len ? std::make_pair(blk[i].off & ~static_cast<uint64_t>(15), blk[i].off + blk[i].len)
                      : std::make_pair(UINT64_MAX, uint64_t{0});
  });
  for (size_t k = 0; k < g.size() && k < cap; ++k) {
    if (first) first[k] = g[k].first;
    if (dev) dev[k] = g[k].dev;
  }
  return static_cast<int64_t>(g.size());
}

}  // namespace
}  // namespace pdb

using namespace pdb;

extern "C" {

int pdb_crc32c_abi_version(void) { return PDB_CRC32C_ABI_VERSION; }

int pdb_host_alloc(uint64_t bytes, void** out) {
  if (!out) return fail(PDB_EINVAL, "null out");
  *out = nullptr;
  if (bytes == 0) return PDB_OK;
  DevState* st;
  int rc = get_state(&st);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  PinAlloc* best = nullptr;  // the smallest kept allocation that fits, within 2x
  for (PinAlloc& a : g_pins)
    if (!a.used && a.cap >= bytes && a.cap / 2 <= bytes && (!best || a.cap < best->cap)) best = &a;
  if (best) {
    best->used = true;
    *out = best->h;
    return PDB_OK;
  }
  g_pin_allocs.fetch_add(1, std::memory_order_relaxed);
  hipError_t e = hipHostMalloc(out, bytes, hipHostMallocDefault);
  if (e != hipSuccess) {
    *out = nullptr;
    return fail(PDB_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
  }
  void* d = nullptr;
  g_pins.push_back(PinAlloc{static_cast<uint8_t*>(*out), hipHostGetDevicePointer(&d, *out, 0) == hipSuccess ? static_cast<uint8_t*>(d) : nullptr,
                            static_cast<size_t>(bytes), true});
  return PDB_OK;
}

int pdb_host_free(void* p) {
  if (!p) return PDB_OK;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  size_t at = g_pins.size();
  for (size_t i = 0; i < g_pins.size(); ++i)
    if (g_pins[i].h == p && g_pins[i].used) at = i;
  if (at == g_pins.size()) return fail(PDB_EINVAL, "pdb_host_free: not a live pdb_host_alloc allocation");
  g_pins[at].used = false;
  hipError_t err = hipSuccess;
  for (;;) {  // release the largest kept allocations while the cache is over either cap
    size_t kept = 0, bytes = 0, big = g_pins.size();
    for (size_t i = 0; i < g_pins.size(); ++i)
      if (!g_pins[i].used) {
        ++kept;
        bytes += g_pins[i].cap;
        if (big == g_pins.size() || g_pins[i].cap > g_pins[big].cap) big = i;
      }
    if (kept <= kPinKeep && bytes <= kPinKeepBytes) break;
    const hipError_t e = hipHostFree(g_pins[big].h);
    if (e != hipSuccess && err == hipSuccess) err = e;
    g_pins.erase(g_pins.begin() + static_cast<std::ptrdiff_t>(big));
  }
  return err == hipSuccess ? PDB_OK : hip_fail(err, "hipHostFree");
}

int pdb_crc32c_init(int device) {
  if (device >= 0) {
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  }
  DevState* st;
  return get_state(&st);
}

int pdb_crc32c_init_mask(uint64_t device_mask) {
  if (device_mask == 0) {
    g_host_mask.store(0, std::memory_order_release);
    return 1;
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0) return fail(PDB_ENODEV, "no HIP device visible (pdb_crc32c has no CPU fallback)");
  if (ndev < 64 && (device_mask >> ndev) != 0) return fail(PDB_EINVAL, "device_mask names a device that is not visible");
  DeviceRestore restore;
  int n = 0;
  for (int d = 0; d < 64; ++d) {
    if (!((device_mask >> d) & 1u)) continue;
    if ((e = hipSetDevice(d)) != hipSuccess) return hip_fail(e, "hipSetDevice");
    DevState* st;
    int rc = get_state(&st);  // the device's tables and contexts, made now
    if (rc) return rc;
    ++n;
  }
  g_host_mask.store(device_mask, std::memory_order_release);
  return n;
}

int64_t pdb_host_stripe_plan(const pdb_blk* blk, uint64_t nblk, uint32_t ndev, uint64_t chunk_bytes, uint64_t* group_first,
                             uint32_t* group_dev, uint64_t cap) {
  if (nblk && !blk) return fail(PDB_EINVAL, "null blocks");
  return stripe_plan(blk, nblk, ndev, chunk_bytes, group_first, group_dev, cap);
}

int pdb_crc32c_prepare_stream(void* stream) {
  DevState* st;
  int rc = get_state(&st);
  if (rc) return rc;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e = hipStreamIsCapturing(s, &cs);
  if (e != hipSuccess) return hip_fail(e, "hipStreamIsCapturing");
  if (cs != hipStreamCaptureStatusNone) return fail(PDB_EINVAL, "pdb_crc32c_prepare_stream: the stream is capturing");
  LongLane ll;
  if (!stream_lane(st, s, &ll)) return fail(PDB_ENOMEM, "no long-block lane for this stream (" + g_err + ")");
  return PDB_OK;
}

const char* pdb_last_error(void) { return g_err.c_str(); }

int pdb_crc32c_current_device(void) {
  int d = -1;
  if (hipGetDevice(&d) != hipSuccess) return -1;
  return d;
}

uint32_t pdb_crc32c_mask(uint32_t crc) { return pdb_mask(crc); }
uint32_t pdb_crc32c_unmask(uint32_t m) { return pdb_unmask(m); }

uint32_t pdb_crc32c_extend(uint32_t init_crc, const void* data, size_t n) {
  if (n == 0) return init_crc;  // Extend over nothing is the identity (util/crc32c.cc:25-32)
  uint32_t out = 0;
  int rc;
  if (n >= kSpanHostThreshold) {  // long span: split across waves, combined on the device
    rc = host_span(init_crc, static_cast<const uint8_t*>(data), n, &out);
  } else {
    rc = host_scalar(init_crc, static_cast<const uint8_t*>(data), n, &out);
  }
  if (rc) {
    fprintf(stderr, "pdb_crc32c_extend: device CRC failed (%d): %s\n", rc, g_err.c_str());
    abort();
  }
  return out;
}

uint32_t pdb_crc32c_value(const void* data, size_t n) { return pdb_crc32c_extend(0, data, n); }

uint64_t pdb_crc32c_extend_scratch_words(uint64_t n) { return span_scratch_words(n); }

int pdb_crc32c_extend_device(uint32_t init_crc, const void* d_data, uint64_t n, uint32_t* d_scratch,
                             uint64_t scratch_words, uint32_t* d_out, void* stream) {
  if (!d_out || (n && !d_data)) return fail(PDB_EINVAL, "null argument");
  if (n > kSpanMaxBytes) return fail(PDB_ERANGE, "span longer than 2^45 bytes");
  if (!d_scratch || scratch_words < span_scratch_words(n))
    return fail(PDB_EINVAL, "scratch smaller than pdb_crc32c_extend_scratch_words(n)");
  DevState* st;
  int rc = get_state(&st);
  if (rc) return rc;
  if ((rc = quiesce(st))) return rc;
  hipError_t e = launch_span(st->geom, st->d_tables, st->d_pow2, init_crc, static_cast<const uint8_t*>(d_data),
                             n, d_scratch, d_out, pick_stream(st, stream));
  return e == hipSuccess ? PDB_OK : hip_fail(e, "launch_span");
}

int pdb_crc32c_batch_device_fixed(const void* d_base, uint64_t stride, uint32_t len, uint64_t nblk,
                                  uint32_t flags, uint32_t init, uint32_t* d_out, void* stream) {
  if (nblk == 0) return PDB_OK;
  if (!d_base || !d_out) return fail(PDB_EINVAL, "null argument");
  DevState* st;
  int rc = get_state(&st);
  if (rc) return rc;
  if ((rc = quiesce(st))) return rc;
  hipError_t e = launch_fixed(st->geom, st->d_tables, static_cast<const uint8_t*>(d_base), stride, len,
                              nblk, flags, init, d_out, pick_stream(st, stream));
  return e == hipSuccess ? PDB_OK : hip_fail(e, "launch_fixed");
}

int pdb_crc32c_batch_device(const void* d_base, const pdb_blk* d_blk, uint64_t nblk, uint32_t flags,
                            uint32_t* d_out, void* stream) {
  if (nblk == 0) return PDB_OK;
  if (!d_base || !d_blk || !d_out) return fail(PDB_EINVAL, "null argument");
  DevState* st;
  int rc = get_state(&st);
  if (rc) return rc;
  if ((rc = quiesce(st))) return rc;
  const hipStream_t s = pick_stream(st, stream);
  LongLane ll;
  hipError_t e = launch_desc(st->geom, st->d_tables, static_cast<const uint8_t*>(d_base), d_blk, nblk,
                             flags, kModeOut, nullptr, d_out, nullptr, nullptr, s, stream_lane(st, s, &ll));
  return e == hipSuccess ? PDB_OK : hip_fail(e, "launch_desc");
}

int pdb_crc32c_verify_device(const void* d_base, const pdb_blk* d_blk, uint64_t nblk, uint32_t flags,
                             const uint32_t* d_expected, uint8_t* d_ok, uint32_t* d_nbad,
                             void* stream) {
  if (nblk == 0) return PDB_OK;
  if (!d_base || !d_blk || !d_expected) return fail(PDB_EINVAL, "null argument");
  DevState* st;
  int rc = get_state(&st);
  if (rc) return rc;
  if ((rc = quiesce(st))) return rc;
  const hipStream_t s = pick_stream(st, stream);
  LongLane ll;
  hipError_t e = launch_desc(st->geom, st->d_tables, static_cast<const uint8_t*>(d_base), d_blk, nblk,
                             flags, kModeVerify, d_expected, nullptr, d_ok, d_nbad, s, stream_lane(st, s, &ll));
  return e == hipSuccess ? PDB_OK : hip_fail(e, "launch_desc(verify)");
}

int pdb_crc32c_batch_host(const void* base, uint64_t base_len, const pdb_blk* blk, uint64_t nblk,
                          uint32_t flags, uint32_t* out) {
  if (nblk && !out) return fail(PDB_EINVAL, "null out");
  return host_desc(static_cast<const uint8_t*>(base), base_len, blk, nblk, flags, kModeOut, nullptr,
                   out, nullptr, nullptr);
}

int64_t pdb_crc32c_verify_host(const void* base, uint64_t base_len, const pdb_blk* blk, uint64_t nblk,
                               uint32_t flags, const uint32_t* expected, uint8_t* ok) {
  if (nblk && !expected) return fail(PDB_EINVAL, "null expected");
  uint64_t nbad = 0;
  const int rc = host_desc(static_cast<const uint8_t*>(base), base_len, blk, nblk, flags, kModeVerify, expected,
                           nullptr, ok, &nbad);
  return rc ? rc : static_cast<int64_t>(nbad);
}

int pdb_sst_seal_device(void* d_buf, uint64_t buf_len, const pdb_block_handle* d_h, uint64_t n,
                        void* stream) {
  if (n == 0) return PDB_OK;
  if (!d_buf || !d_h) return fail(PDB_EINVAL, "null argument");
  // a handle whose block + trailer leaves the buffer is reported bad (verify) or skipped (seal)
  // by the kernel; below one trailer there is no valid handle at all
  if (buf_len < 5) return fail(PDB_ERANGE, "buffer smaller than one block trailer");
  DevState* st;
  int rc = get_state(&st);
  if (rc) return rc;
  if ((rc = quiesce(st))) return rc;
  const hipStream_t s = pick_stream(st, stream);
  LongLane ll;
  hipError_t e = launch_sst(st->geom, st->d_tables, static_cast<uint8_t*>(d_buf), buf_len, d_h, n, true,
                            nullptr, nullptr, s, stream_lane(st, s, &ll));
  return e == hipSuccess ? PDB_OK : hip_fail(e, "launch_sst(seal)");
}

int pdb_sst_verify_device(const void* d_buf, uint64_t buf_len, const pdb_block_handle* d_h,
                          uint64_t n, uint8_t* d_ok, uint32_t* d_nbad, void* stream) {
  if (n == 0) return PDB_OK;
  if (!d_buf || !d_h) return fail(PDB_EINVAL, "null argument");
  // a handle whose block + trailer leaves the buffer is reported bad (verify) or skipped (seal)
  // by the kernel; below one trailer there is no valid handle at all
  if (buf_len < 5) return fail(PDB_ERANGE, "buffer smaller than one block trailer");
  DevState* st;
  int rc = get_state(&st);
  if (rc) return rc;
  if ((rc = quiesce(st))) return rc;
  const hipStream_t s = pick_stream(st, stream);
  LongLane ll;
  hipError_t e = launch_sst(st->geom, st->d_tables, static_cast<uint8_t*>(const_cast<void*>(d_buf)),
                            buf_len, d_h, n, false, d_ok, d_nbad, s, stream_lane(st, s, &ll));
  return e == hipSuccess ? PDB_OK : hip_fail(e, "launch_sst(verify)");
}

int pdb_sst_crc_device(const void* d_buf, uint64_t buf_len, const pdb_block_handle* d_h, uint64_t n,
                       uint32_t* d_out, void* stream) {
  if (n == 0) return PDB_OK;
  if (!d_buf || !d_h || !d_out) return fail(PDB_EINVAL, "null argument");
  if (buf_len < 5) return fail(PDB_ERANGE, "buffer smaller than one block trailer");
  DevState* st;
  int rc = get_state(&st);
  if (rc) return rc;
  if ((rc = quiesce(st))) return rc;
  const hipStream_t s = pick_stream(st, stream);
  LongLane ll;
  hipError_t e = launch_sst_masked(st->geom, st->d_tables, static_cast<uint8_t*>(const_cast<void*>(d_buf)), buf_len,
                                   d_h, n, d_out, s, stream_lane(st, s, &ll));
  return e == hipSuccess ? PDB_OK : hip_fail(e, "launch_sst_masked");
}

int pdb_sst_seal_host(void* buf, uint64_t buf_len, const pdb_block_handle* h, uint64_t n) {
  return host_sst(static_cast<uint8_t*>(buf), buf_len, h, n, true, nullptr, nullptr);
}

int64_t pdb_sst_verify_host(const void* buf, uint64_t buf_len, const pdb_block_handle* h, uint64_t n,
                            uint8_t* ok) {
  int64_t nbad = 0;
  int rc = host_sst(static_cast<uint8_t*>(const_cast<void*>(buf)), buf_len, h, n, false, ok, &nbad);
  return rc ? rc : nbad;
}

}  // extern "C"
