// tools/lds_probe.hip -- LDS read forms on gfx950 (diagnostics only): do ds_read_b64 / ds_read_b128
// at 4-B (not naturally) aligned addresses return the right bytes, and what do they cost per
// wave-instruction next to the aligned forms and ds_read_b32 / ds_read2_b32?
//
// One 1024-thread workgroup per CU (16 waves), each wave reading its own 4-KiB window of a 64-KiB
// LDS image: lane u reads at dword stride*u + mis (+ a multiple of 64 dwords per independent read,
// which keeps the bank pattern).  16 reads in flight per loop iteration; s_memtime around the loop
// gives shader cycles; cycles per wave-instruction per CU = cycles / (16 waves x reads).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_lds_probe tools/lds_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
      return 1;                                                         \
    }                                                                   \
  } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));

constexpr uint32_t kLdsWords = 16384;  // 64 KiB
constexpr int kIters = 256, kInner = 16;

__device__ __forceinline__ uint32_t pat(uint32_t i) { return i * 0x9E3779B9u ^ (i >> 7); }

// W: 1 = b32, 2 = b64 (declared 8-B aligned), 3 = read2_b32 (8 B declared 4-B aligned), 4 = b128
template <int W>
__global__ __launch_bounds__(1024) void probe(uint32_t stride, uint32_t mis, uint32_t* out, uint64_t* cyc, uint32_t check) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
  for (uint32_t i = threadIdx.x; i < kLdsWords; i += blockDim.x) lds[i] = pat(i);
  __syncthreads();
  const uint32_t u = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t base = (wv * 1024u + stride * u + mis) & (kLdsWords - 1u);  // dwords
  if (check) {  // one read per lane: the bytes it returned
    const char* p = reinterpret_cast<const char*>(lds) + 4u * base;
    uint32_t v[4] = {0, 0, 0, 0};
    if constexpr (W == 1) v[0] = *reinterpret_cast<const uint32_t*>(p);
    if constexpr (W == 2) { const u32x2 x = *reinterpret_cast<const u32x2*>(p); v[0] = x.x; v[1] = x.y; }
    if constexpr (W == 3) { const u32x2a4 x = *reinterpret_cast<const u32x2a4*>(p); v[0] = x.x; v[1] = x.y; }
    if constexpr (W == 4) { const u32x4 x = *reinterpret_cast<const u32x4*>(p); v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; }
    if (blockIdx.x == 0)
      for (int k = 0; k < 4; ++k) out[4u * threadIdx.x + k] = v[k];
    return;
  }
  uint32_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
    uint32_t r[kInner];
#pragma unroll
    for (int k = 0; k < kInner; ++k) {
      const uint32_t a = (base + 64u * ((k + it) & 15u)) & (kLdsWords - 1u);
      const char* p = reinterpret_cast<const char*>(lds) + 4u * a;
      if constexpr (W == 1) r[k] = *reinterpret_cast<const uint32_t*>(p);
      if constexpr (W == 2) { const u32x2 x = *reinterpret_cast<const u32x2*>(p); r[k] = x.x ^ x.y; }
      if constexpr (W == 3) { const u32x2a4 x = *reinterpret_cast<const u32x2a4*>(p); r[k] = x.x ^ x.y; }
      if constexpr (W == 4) { const u32x4 x = *reinterpret_cast<const u32x4*>(p); r[k] = (x.x ^ x.y) ^ (x.z ^ x.w); }
    }
#pragma unroll
    for (int k = 0; k < kInner; ++k) acc = acc * 3u + r[k];
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  if (acc == 0x12345678u) out[0] = acc;  // keep the reads
}

template <int W>
int run(const char* name, uint32_t stride, uint32_t mis, int ncu, uint32_t* d_out, uint64_t* d_cyc) {
  // correctness: the returned words must be pat(base .. base + words - 1)
  CK(hipMemset(d_out, 0, 4096 * 4));
  hipLaunchKernelGGL(probe<W>, dim3(1), dim3(1024), 0, 0, stride, mis, d_out, d_cyc, 1u);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> h(4096);
  CK(hipMemcpy(h.data(), d_out, 4096 * 4, hipMemcpyDeviceToHost));
  const int words = W == 1 ? 1 : (W == 4 ? 4 : 2);
  int bad = 0;
  for (uint32_t t = 0; t < 1024; ++t) {
    const uint32_t u = t & 63u, wv = t >> 6;
    const uint32_t base = (wv * 1024u + stride * u + mis) & (kLdsWords - 1u);
    for (int k = 0; k < words; ++k) {
      const uint32_t i = base + k;
      if (h[4 * t + k] != (i * 0x9E3779B9u ^ (i >> 7))) ++bad;
    }
  }
  // timing: every CU, 3 launches, the last one counted
  std::vector<uint64_t> c(ncu);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe<W>, dim3(ncu), dim3(1024), 0, 0, stride, mis, d_out, d_cyc, 0u);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(c.data(), d_cyc, ncu * 8, hipMemcpyDeviceToHost));
  double mean = 0;
  for (int i = 0; i < ncu; ++i) mean += c[i];
  mean /= ncu;
  const double instr = 16.0 * kIters * kInner;  // wave-instructions per CU
  printf("{\"form\": \"%s\", \"stride\": %u, \"mis\": %u, \"bad_words\": %d, \"cycles_per_wave_instr\": %.3f, "
         "\"bytes_per_cycle_per_cu\": %.1f}\n",
         name, stride, mis, bad, mean / instr, 64.0 * 4 * words * instr / mean);
  return 0;
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t* d_out;
  uint64_t* d_cyc;
  CK(hipMalloc(&d_out, 4096 * 4));
  CK(hipMalloc(&d_cyc, ncu * 8));
  run<1>("ds_read_b32", 1, 0, ncu, d_out, d_cyc);
  run<1>("ds_read_b32", 2, 0, ncu, d_out, d_cyc);  // 2-way
  run<3>("ds_read2_b32 (8 B at 4-B alignment)", 2, 0, ncu, d_out, d_cyc);
  run<3>("ds_read2_b32 (8 B at 4-B alignment)", 2, 1, ncu, d_out, d_cyc);
  run<2>("ds_read_b64", 2, 0, ncu, d_out, d_cyc);
  run<2>("ds_read_b64", 2, 1, ncu, d_out, d_cyc);
  run<2>("ds_read_b64", 3, 0, ncu, d_out, d_cyc);
  run<2>("ds_read_b64", 3, 1, ncu, d_out, d_cyc);
  run<2>("ds_read_b64", 1, 0, ncu, d_out, d_cyc);
  run<2>("ds_read_b64", 1, 1, ncu, d_out, d_cyc);
  run<4>("ds_read_b128", 4, 0, ncu, d_out, d_cyc);
  run<4>("ds_read_b128", 4, 1, ncu, d_out, d_cyc);
  run<4>("ds_read_b128", 4, 2, ncu, d_out, d_cyc);
  run<4>("ds_read_b128", 5, 0, ncu, d_out, d_cyc);
  run<4>("ds_read_b128", 5, 1, ncu, d_out, d_cyc);
  run<4>("ds_read_b128", 1, 0, ncu, d_out, d_cyc);
  run<4>("ds_read_b128", 1, 3, ncu, d_out, d_cyc);
  return 0;
}
