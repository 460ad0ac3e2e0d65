// crc32c_server.hip -- the scalar Extend service: a persistent one-workgroup kernel that serves
// leveldb::crc32c::Extend calls (util/crc32c.h:17; called per WAL record by log_writer.cc:121,
// per sstable block by table_builder.cc:197-199 and format.cc:97) from request slots in a mailbox.
//
// Why: a synchronous scalar call is latency-bound.  Launching a kernel per call costs ~10 us
// (dispatch, wave launch, staging the 160-KiB LDS image, PCIe reads, result write;
// profiles/r01_scalar_latency_poll.json).  The server pays dispatch and LDS staging once per
// lifetime and then only polls its mailbox, reads the caller's bytes, hashes them with one wave
// and posts the CRC back across PCIe.
//
// Protocol (crc32c_internal.h): kServerSlots request slots, each with its own request word
// {init, len, seq} and data area; a caller thread owns a slot (no global lock on the host), writes
// its bytes (placed so that they END on a 16-B boundary) and then the request word, and spins on
// its slot's response word {crc, seq}.  The workgroup's kServerWaves waves each poll a quarter of
// the slots with ONE vector load (lane l: slot w + 16 l) and serve the lowest pending one, so up
// to kServerWaves requests are hashed at once.  A request is pending while its req seq differs
// from its resp seq: an instance initialises its view from the resp words, so requests posted
// while no instance was polling are served by the next one.  The instance leaves when ctl->stop
// changes, after `idle_ticks` without a request in ANY slot, or after `life_ticks` in total
// (s_memrealtime, 100 MHz): the first wave to see the condition sets a closing flag in LDS, every
// wave leaves at its next poll without serving, and the last one out writes exit_epoch = its
// epoch, so the host can tell a live server from a finished one without a HIP call.
//
// Per request, a wave hashes n bytes with the geometry of crc_stream16_kernel (16-B lane pieces,
// rounds of 4 KiB: piece c = 256r + 64j + u on lane u, chain j; 4 chains folded with shift 1024,
// rounds chained with shift 1008, rotation by K mod 64, 6-level DPP tree over 16 << k), with every
// piece 16-B aligned by the host's placement; the t = n mod 16 head bytes are hashed from the
// seed on broadcast words.  Loads of up to 4 rounds (16 KiB) are issued together so a request
// pays about one memory round trip per 16 KiB.
#include "crc32c_device.h"

namespace pdb {
namespace {

__device__ __forceinline__ uint64_t sys_load64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void sys_store64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void sys_store32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// System-coherent 16-B load (sc0 sc1: bypasses the GPU caches, so bytes the host wrote into a
// mailbox in host memory or in fine-grained device memory are never served stale from L2).
__device__ __forceinline__ u32x4 ld_sys16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 17));
}

__device__ __forceinline__ uint32_t u4(const u32x4& v, uint32_t i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

// Raw state after the n bytes at byte offset data_off of the request box from state init_raw;
// valid in lane 0.  q0 = data_off + n % 16 is 16-B aligned and the head (n % 16 bytes) is the tail
// of the aligned 16 B before q0.  Every load of a 16-KiB batch is issued unconditionally
// (out-of-range pieces read q0 - 16 and are ignored), so a batch costs one memory round trip.
__device__ __forceinline__ uint32_t server_hash(const char* lds, const LaneTabs& lt, uint32_t u,
                                                __amdgpu_buffer_rsrc_t rin, uint32_t data_off, uint32_t n,
                                                uint32_t init_raw) {
  const uint32_t t = n & 15u, lead = t & 3u, nh = t >> 2, K = n >> 4;
  const uint32_t q0 = data_off + t;
  const uint32_t R = (K + 255u) >> 8;
  uint32_t acc = 0, h = init_raw;
  for (uint32_t r0 = 0; r0 < R || r0 == 0; r0 += 4) {
    u32x4 e[4][4];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t c = ((r0 + rr) << 8) + 64u * j + u;
        e[rr][j] = ld_sys16(rin, c < K ? q0 + 16u * c : q0 - 16u);
      }
    if (r0 == 0) {
      // head: dwords 4-nh..3 of the 16 B before q0, preceded by the top `lead` bytes of dword 3-nh
      const u32x4 hv = ld_sys16(rin, q0 - 16u);
      if (lead) {
        const uint32_t lb = u4(hv, 3u - nh) >> (8u * (4u - lead));
        for (uint32_t j = 0; j < lead; ++j) h = step1(lds, lt, h, (lb >> (8u * j)) & 0xffu);
      }
      for (uint32_t j = 4u - nh; j < 4u; ++j) h = step4(lds, lt, h, u4(hv, j));
      acc = u == 0 ? h : 0u;
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const uint32_t ck = r0 + rr;
      if (ck >= R) break;  // wave-uniform
      const uint32_t rem = K - (ck << 8);
      const uint32_t J = rem >= 256u ? 4u : (rem > u ? ((rem - u - 1u) >> 6) + 1u : 0u);
      if (J) {
        const uint32_t start = ck ? shift_op(lds, PDB_SLOT_HORNER, acc) : acc;
        const uint32_t x0 = chain16(lds, lt, start, e[rr][0], 0u, 0u);
        const uint32_t x1 = chain16(lds, lt, 0u, e[rr][1], 0u, 0u);
        const uint32_t x2 = chain16(lds, lt, 0u, e[rr][2], 0u, 0u);
        const uint32_t x3 = chain16(lds, lt, 0u, e[rr][3], 0u, 0u);
        uint32_t a = x0;
        if (J > 1) a = shift_op_x(lds, 7, a, x1);
        if (J > 2) a = shift_op_x(lds, 7, a, x2);
        if (J > 3) a = shift_op_x(lds, 7, a, x3);
        acc = a;
      }
    }
  }
  if (K == 0) return h;
  const uint32_t q = K & 63u;
  if (q) acc = __shfl(acc, (u + q) & 63u, 64);
  return wave_tree_dpp<true>(lds, u, acc);  // slot 5 holds the workgroup state
}

__global__ __launch_bounds__(64 * kServerWaves) void crc_server_kernel(const uint32_t* __restrict__ tabs,
                                                                        uint8_t* in, uint8_t* out, uint32_t epoch,
                                                                        uint64_t stop0, uint64_t idle_ticks,
                                                                        uint64_t life_ticks, uint32_t stamps) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[PDB_LDS_BYTES / 4];
  char* lds = reinterpret_cast<char*>(lds_words);
  // operator slot 5 stays free (tree level 5 = shift 256 twice) and holds the workgroup's state
  stage_tables<PDB_CAT_TREE16, PDB_CAT_H1008, PDB_CAT_S1024, /*kSkipSlot5=*/true>(lds, tabs);
  uint32_t* wg = reinterpret_cast<uint32_t*>(lds + PDB_MAIN_BYTES + 5u * 4096u);
  // wg[0] closing, wg[1] waves out, wg[2] requests, wg[3] polls (low 32 bits), wg[4..5] last
  // request tick, wg[6..7] serve ticks
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    wg[0] = 0u;
    wg[1] = 0u;
    wg[2] = 0u;
    wg[3] = 0u;
    *reinterpret_cast<uint64_t*>(wg + 4) = t0;
    *reinterpret_cast<uint64_t*>(wg + 6) = 0u;
  }
  __syncthreads();
  const uint32_t u = threadIdx.x & 63u;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const LaneTabs lt = lane_tabs(u);
  const __amdgpu_buffer_rsrc_t rin =
      __builtin_amdgcn_make_buffer_rsrc(in, 0, static_cast<int>(kServerInBytes), 0x00020000);
  constexpr uint32_t kPer = kServerSlots / kServerWaves;  // slots per wave
  const uint32_t slot = w + kServerWaves * (u < kPer ? u : 0u);
  const uint64_t* req = reinterpret_cast<const uint64_t*>(in + kReqOff);
  // the seq each slot last had answered, from the response words (pinned host memory)
  uint32_t served = static_cast<uint32_t>(sys_load64(reinterpret_cast<const uint64_t*>(out + 64u * slot)) >> 32) &
                    kServerSeqMask;
  const ServerCtl* ctl = reinterpret_cast<const ServerCtl*>(in);
  uint64_t t_last = t0, serve_ticks = 0;
  uint32_t n_req = 0, n_poll = 0;
  // Two polls in flight: the next poll's loads are issued before the current one is examined (the
  // loop is unrolled over two register sets, so no copy of a result in flight forces a wait), and a
  // request is seen about half a memory round trip sooner (a poll of fine-grained device memory is a
  // full round trip).  A poll issued before an answer was posted still shows the answered seq, so it
  // is never mistaken for a new request.
  auto poll_step = [&](const uint64_t rq, const uint64_t stop) -> bool {  // true: leave
    ++n_poll;
    const uint32_t seq_l = static_cast<uint32_t>(rq >> 49);
    const uint64_t pend = __builtin_amdgcn_ballot_w64(u < kPer && seq_l != served);
    const bool closing = __hip_atomic_load(wg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u;
    if (closing || __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(stop)) != static_cast<uint32_t>(stop0) ||
        __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(stop >> 32)) != static_cast<uint32_t>(stop0 >> 32))
      return true;
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (pend) {
      // no acquire fence: every load of the request bytes is system-coherent (sc0 sc1) and is
      // issued only after this poll returned (control dependency), so it sees the bytes the host
      // wrote before the request word (x86 store order + sfence, PCIe posted-write order)
      const uint32_t l = static_cast<uint32_t>(__builtin_ctzll(pend));
      const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(rq >> 32), l);
      const uint32_t init = __builtin_amdgcn_readlane(static_cast<uint32_t>(rq), l);
      const uint32_t sq = hi >> 17, n = hi & 0x1FFFFu;
      const uint32_t s_srv = w + kServerWaves * l;
      uint32_t crc = 0;
      if (n <= kServerCap) {  // (a malformed length is answered with 0 rather than read out of range)
        const uint32_t data_off = static_cast<uint32_t>(kSlotDataOff + s_srv * kSlotStride) + ((0u - n) & 15u);
        crc = ~server_hash(lds, lt, u, rin, data_off, n, ~init);
      }
      // phase stamps (PDB_SERVER_STAMPS, diagnostics: tools/scalar_phases.py): the tick at which the
      // poll that found the request returned and the tick after the hash, in the response line's
      // words 1 and 2, written before the response word (the host reads them once it sees it)
      if (stamps && u == 0) {
        uint64_t* line = reinterpret_cast<uint64_t*>(out + 64u * s_srv);
        sys_store64(line + 1, now);
        sys_store64(line + 2, __builtin_amdgcn_s_memrealtime());
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      }
      if (u == 0) sys_store64(reinterpret_cast<uint64_t*>(out + 64u * s_srv), (static_cast<uint64_t>(sq) << 32) | crc);
      if (u == l) served = sq;
      t_last = now;
      if (u == 0) *reinterpret_cast<uint64_t*>(wg + 4) = now;  // any wave's request keeps all alive
      ++n_req;
      serve_ticks += __builtin_amdgcn_s_memrealtime() - now;
      return false;
    }
    // idle: the workgroup's last-request tick is read only once this wave's own is older than the
    // idle limit (a read of it on every poll made the compiler drain the polls in flight)
    if (now - t_last > idle_ticks || now - t0 > life_ticks) {
      const uint64_t last = __hip_atomic_load(reinterpret_cast<uint64_t*>(wg + 4), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
      if (last > t_last) t_last = last;  // another wave served since
      if (now - t_last > idle_ticks || now - t0 > life_ticks) {
        if (u == 0) __hip_atomic_store(wg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return true;
      }
    }
    __builtin_amdgcn_s_sleep(2);
    return false;
  };
  uint64_t rqA = sys_load64(req + slot), stA = sys_load64(&ctl->stop);
  for (;;) {
    const uint64_t rqB = sys_load64(req + slot), stB = sys_load64(&ctl->stop);
    if (poll_step(rqA, stA)) break;
    rqA = sys_load64(req + slot);
    stA = sys_load64(&ctl->stop);
    if (poll_step(rqB, stB)) break;
  }
  // the last wave out publishes the exit (and the counters)
  uint32_t out_before = 0;
  if (u == 0) {
    __hip_atomic_fetch_add(wg + 2, n_req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_add(wg + 3, n_poll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(wg + 6), static_cast<unsigned long long>(serve_ticks),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    out_before = __hip_atomic_fetch_add(wg + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  out_before = __builtin_amdgcn_readfirstlane(out_before);
  if (out_before + 1u == kServerWaves && u == 0) {
    ServerExit* ex = reinterpret_cast<ServerExit*>(out + kExitOff);
    sys_store64(&ex->stat_requests, __hip_atomic_load(wg + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    sys_store64(&ex->stat_serve_ticks, __hip_atomic_load(reinterpret_cast<unsigned long long*>(wg + 6),
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    sys_store64(&ex->stat_polls, __hip_atomic_load(wg + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    sys_store64(&ex->stat_life_ticks, __builtin_amdgcn_s_memrealtime() - t0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    sys_store32(&ex->exit_epoch, epoch);
  }
}

}  // namespace

hipError_t launch_server(const uint32_t* d_tables, uint8_t* d_in, uint8_t* d_out, uint32_t epoch, uint64_t stop0,
                         uint64_t idle_ticks, uint64_t life_ticks, uint32_t stamps, hipStream_t s) {
  hipLaunchKernelGGL(crc_server_kernel, dim3(1), dim3(64 * kServerWaves), 0, s, d_tables, d_in, d_out, epoch, stop0,
                     idle_ticks, life_ticks, stamps);
  return hipGetLastError();
}

}  // namespace pdb
