// tools/dma_inflight.hip -- diagnostics (never linked into the product): HBM read rate of a wave
// pipeline that stages 1-KiB-contiguous chunks through LDS, by how the chunks get there and how many
// bytes a CU keeps in flight.  The question it answers: can the
// record kernel (crc_lanespan_kernel) gain by staging its spans with gfx950 LDS-DMA
// (global_load_lds_dwordx4) instead of registers + ds_write_b128?  A DMA has no register stage, so
// every byte in flight occupies LDS, and the record kernel has 96 KiB of LDS beside its tables for
// everything: the item being hashed AND the items in flight.  Register staging keeps its in-flight
// items in VGPRs (11 waves x 2 items x 9 KiB today).  This kernel does no hashing at all: each wave
// cycles S slots of J KiB, waits for the oldest, reads one dword per lane per KiB of it and reissues
// the slot, so the rate it reports is a ceiling for any kernel with that much in flight.
//
//   dma:  J global_load_lds_dwordx4 per item (64 lanes x 16 B = 1 KiB each) into the slot, M0 = the
//         slot's LDS address; waits by explicit vmcnt (inline asm: the compiler's own waitcnt pass
//         would wait for every DMA before any read of the same LDS object)
//   reg:  J global_load_dwordx4 (nt) per item into registers, S items in flight, then J ds_write_b128
//         into the wave's slot (the record kernel's issue() / to_lds())
//
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/dma_inflight.hip -o tools/_build/dma_inflight
// usage: dma_inflight [GiB=4] [launches=20]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// one 1-KiB chunk: lane u's 16 B at g + 16 u land at LDS byte m0 + 16 u
__device__ __forceinline__ void dma_chunk(const uint8_t* g, uint32_t m0) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}

// W waves per workgroup, one workgroup per CU (the dynamic LDS below keeps it so), J KiB per item,
// S slots per wave.  Wave w of the grid takes items w, w + G, ... (G = waves in the grid).
template <int W, int J, int S, bool kDma>
__global__ __launch_bounds__(W * 64) void stage_kernel(const uint8_t* __restrict__ buf, uint64_t nitems, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t u = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t G = static_cast<uint64_t>(gridDim.x) * W;
  const uint64_t first = static_cast<uint64_t>(blockIdx.x) * W + wv;
  constexpr uint32_t kWaveBytes = (kDma ? S : 1) * J * 1024u;  // register staging: one region per wave
  uint8_t* region = lds + wv * kWaveBytes;
  const uint32_t rbase = wv * kWaveBytes;  // LDS byte address (the dynamic array starts at 0: no static LDS)
  uint32_t acc = 0;
  auto consume = [&](uint32_t s) {
#pragma unroll
    for (int j = 0; j < J; ++j) acc ^= *reinterpret_cast<const uint32_t*>(region + s * J * 1024u + 1024u * j + 16u * u);
  };
  if constexpr (kDma) {
    auto issue = [&](uint32_t s, uint64_t it) {
      const uint8_t* g = buf + it * (J * 1024ull) + 16u * u;
#pragma unroll
      for (int j = 0; j < J; ++j) dma_chunk(g + 1024u * j, __builtin_amdgcn_readfirstlane(rbase + s * J * 1024u + 1024u * j));
    };
    // prologue: S items in flight (past the end: re-read item `first`, never consumed)
    uint64_t it = first;
#pragma unroll
    for (int s = 0; s < S; ++s) issue(s, it + s * G < nitems ? it + s * G : first);
    for (uint32_t s = 0; it < nitems; it += G, s = (s + 1 == S ? 0 : s + 1)) {
      wait_vm<(S - 1) * J>();  // the oldest slot has landed
      consume(s);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // its reads done before the slot is reloaded
      const uint64_t nx = it + S * G;
      issue(s, nx < nitems ? nx : first);
    }
    wait_vm<0>();
  } else {
    u32x4 A[S][J];
    auto issue = [&](u32x4 (&a)[J], uint64_t it) {
      const u32x4* g = reinterpret_cast<const u32x4*>(buf + it * (J * 1024ull) + 16u * u);
#pragma unroll
      for (int j = 0; j < J; ++j) a[j] = __builtin_nontemporal_load(g + 64u * j);
    };
    uint64_t it = first;
#pragma unroll
    for (int s = 0; s < S; ++s) issue(A[s], it + s * G < nitems ? it + s * G : first);
    // rotate the register arrays by full unrolling of one round of S items
    for (; it < nitems;) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (it >= nitems) break;
#pragma unroll
        for (int j = 0; j < J; ++j) *reinterpret_cast<u32x4*>(region + 1024u * j + 16u * u) = A[s][j];
        const uint64_t nx = it + S * G;
        issue(A[s], nx < nitems ? nx : first);
        consume(0);
        it += G;
      }
    }
  }
  if (acc == 0x9E3779B9u) out[0] = acc;  // keep the reads
}

struct Cfg {
  const char* name;
  void (*launch)(const uint8_t*, uint64_t, uint32_t*, uint32_t, hipStream_t);
  int waves, J, S;
  bool dma;
};

template <int W, int J, int S, bool kDma>
void launch_cfg(const uint8_t* buf, uint64_t bytes, uint32_t* out, uint32_t cus, hipStream_t st) {
  const uint64_t nitems = bytes / (J * 1024ull);
  const size_t lds = static_cast<size_t>(W) * (kDma ? S : 1) * J * 1024u;
  // at least 96 KiB of LDS per workgroup (one workgroup per CU, as the record kernel)
  const size_t dyn = lds < (96u << 10) ? (96u << 10) : lds;
  static bool attr = false;
  if (!attr) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(stage_kernel<W, J, S, kDma>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(dyn)));
    attr = true;
  }
  hipLaunchKernelGGL((stage_kernel<W, J, S, kDma>), dim3(cus), dim3(W * 64), dyn, st, buf, nitems, out);
}

int main(int argc, char** argv) {
  const uint64_t gib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 4;
  const int launches = argc > 2 ? atoi(argv[2]) : 20;
  const uint64_t bytes = gib << 30;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const uint32_t cus = prop.multiProcessorCount;
  uint8_t* buf;
  uint32_t* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 256));
  CK(hipMemset(buf, 0x5B, bytes));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  // in flight per CU (KiB) = waves x S x J for a loads-only pipeline; a hashing kernel holds one of
  // its S slots while it hashes, so (S - 1) x J per wave stay in flight then
  static const Cfg cfgs[] = {
      {"reg  11w x 2 x 9 KiB (the record kernel's staging today)", launch_cfg<11, 9, 2, false>, 11, 9, 2, false},
      {"reg  11w x 1 x 9 KiB", launch_cfg<11, 9, 1, false>, 11, 9, 1, false},
      {"reg  11w x 1 x 4 KiB", launch_cfg<11, 4, 1, false>, 11, 4, 1, false},
      {"dma  11w x 2 x 4 KiB (two half-regions: 88 KiB LDS)", launch_cfg<11, 4, 2, true>, 11, 4, 2, true},
      {"dma  11w x 1 x 4 KiB (= one half in flight while the other is hashed)", launch_cfg<11, 4, 1, true>, 11, 4, 1, true},
      {"dma   5w x 2 x 9 KiB (two full regions: 90 KiB LDS)", launch_cfg<5, 9, 2, true>, 5, 9, 2, true},
      {"dma   5w x 1 x 9 KiB (= one region in flight while the other is hashed)", launch_cfg<5, 9, 1, true>, 5, 9, 1, true},
      {"dma  12w x 1 x 8 KiB (all 96 KiB in flight, nothing hashed)", launch_cfg<12, 8, 1, true>, 12, 8, 1, true},
      {"dma  12w x 2 x 4 KiB (all 96 KiB in flight, 2 slots)", launch_cfg<12, 4, 2, true>, 12, 4, 2, true},
      {"dma  16w x 2 x 5 KiB (160 KiB: the whole LDS, no tables)", launch_cfg<16, 5, 2, true>, 16, 5, 2, true},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("{\"tool\": \"dma_inflight\", \"bytes\": %llu, \"cus\": %u, \"launches\": %d, \"rows\": [\n",
         static_cast<unsigned long long>(bytes), cus, launches);
  for (size_t c = 0; c < sizeof(cfgs) / sizeof(cfgs[0]); ++c) {
    const Cfg& f = cfgs[c];
    for (int i = 0; i < 5; ++i) f.launch(buf, bytes, out, cus, st);
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < launches; ++i) f.launch(buf, bytes, out, cus, st);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double per = ms / launches;
    const double tbs = bytes / (per * 1e-3) / 1e12;
    printf("  {\"cfg\": \"%s\", \"dma\": %s, \"waves\": %d, \"slot_KiB\": %d, \"slots\": %d, \"lds_KiB_per_CU\": %d, "
           "\"ms\": %.4f, \"TB_s\": %.3f, \"frac_8TBs\": %.4f}%s\n",
           f.name, f.dma ? "true" : "false", f.waves, f.J, f.S, f.waves * f.J * (f.dma ? f.S : 1), per, tbs, tbs / 8.0,
           c + 1 < sizeof(cfgs) / sizeof(cfgs[0]) ? "," : "");
    fflush(stdout);
  }
  printf("]}\n");
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
