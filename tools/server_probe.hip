// tools/server_probe.hip -- latency calibration for the scalar Extend service (diagnostics only).
//   1. GPU -> host-memory read round trip: one lane chases NSTEP dependent loads through pinned,
//      device-mapped host memory (the mailbox's kind of memory); s_memrealtime brackets them.
//   2. The same chase through fine-grained device memory and ordinary device memory.
//   3. Shader clock while a lone wave spins (s_memtime vs s_memrealtime).
//   4. Host <-> GPU ping-pong through pinned host memory: the host bumps a word, a resident
//      one-wave kernel echoes it back; host-measured round trip per exchange.
//   5. Whether the host can write fine-grained device memory directly (SIGSEGV caught).
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/_server_probe tools/server_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <setjmp.h>
#include <signal.h>
#include <time.h>
#include <unistd.h>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                \
    }                                                                          \
  } while (0)

static double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

constexpr int kSteps = 2000;
static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }

__global__ void chase(const uint32_t* p, uint32_t steps, uint64_t* out) {
  if (threadIdx.x) return;
  uint32_t i = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  for (uint32_t s = 0; s < steps; ++s) i = __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  out[0] = t1 - t0;
  out[1] = c1 - c0;
  out[2] = i;
}

// Echo: wait for host word h[0] to change, write it to h[16]; `n` exchanges, bounded by a deadline.
__global__ void echo(uint32_t* h, uint32_t n, uint64_t deadline_ticks, uint64_t* out) {
  if (threadIdx.x) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t last = 0, done = 0, polls = 0;
  while (done < n) {
    const uint32_t v = __hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    ++polls;
    if (v != last) {
      last = v;
      __hip_atomic_store(h + 16, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      ++done;
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > deadline_ticks) break;
  }
  out[0] = done;
  out[1] = polls;
  out[2] = __builtin_amdgcn_s_memrealtime() - t0;
}

int chase_mem(const char* name, uint32_t* dptr, uint32_t* hinit, bool host_visible, uint64_t* d_out) {
  // ring of kSteps+1 entries with a stride of 64 words (one 256-B line per step)
  const int n = (kSteps + 1) * 64;
  uint32_t* tmp = new uint32_t[n];
  for (int s = 0; s <= kSteps; ++s) tmp[s * 64] = ((s + 1) % (kSteps + 1)) * 64;
  if (host_visible)
    for (int i = 0; i < n; i += 64) hinit[i] = tmp[i];
  else
    CK(hipMemcpy(dptr, tmp, n * 4, hipMemcpyHostToDevice));
  delete[] tmp;
  hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, dptr, kSteps, d_out);
  CK(hipDeviceSynchronize());
  uint64_t r[3];
  CK(hipMemcpy(r, d_out, sizeof(r), hipMemcpyDeviceToHost));
  printf("{\"probe\": \"chase\", \"memory\": \"%s\", \"ns_per_load\": %.1f, \"shader_MHz\": %.0f}\n", name,
         r[0] * 10.0 / kSteps, r[0] ? 100.0 * r[1] / r[0] : 0.0);
  fflush(stdout);
  return 0;
}

int main() {
  uint64_t* d_out;
  CK(hipMalloc(&d_out, 64));
  const size_t bytes = (kSteps + 1) * 256;
  // 1. pinned host memory (what the mailbox uses)
  uint32_t *hp, *hp_d;
  CK(hipHostMalloc(reinterpret_cast<void**>(&hp), bytes, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hp_d), hp, 0));
  if (chase_mem("pinned host (coherent)", hp_d, hp, true, d_out)) return 1;
  // 2. device memory, fine-grained and coarse-grained
  uint32_t* fg = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&fg), bytes, hipDeviceMallocFinegrained));
  if (chase_mem("device fine-grained", fg, nullptr, false, d_out)) return 1;
  uint32_t* cg = nullptr;
  CK(hipMalloc(&cg, bytes));
  if (chase_mem("device coarse-grained", cg, nullptr, false, d_out)) return 1;
  // 4. host <-> GPU ping-pong through pinned host memory
  {
    volatile uint32_t* h = hp;
    h[0] = 0;
    h[16] = 0;
    const uint32_t N = 20000;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(echo, dim3(1), dim3(64), 0, s, hp_d, N, 300000000ull, d_out);
    // wait for the kernel to start polling: first exchange
    double tfirst = now_s();
    h[0] = 1;
    while (h[16] != 1) {
      if (now_s() - tfirst > 5) {
        fprintf(stderr, "echo kernel did not answer\n");
        return 1;
      }
    }
    const double t0 = now_s();
    for (uint32_t k = 2; k <= N; ++k) {
      h[0] = k;
      while (h[16] != k) __builtin_ia32_pause();
    }
    const double dt = now_s() - t0;
    CK(hipStreamSynchronize(s));
    uint64_t r[3];
    CK(hipMemcpy(r, d_out, sizeof(r), hipMemcpyDeviceToHost));
    printf("{\"probe\": \"pingpong\", \"memory\": \"pinned host\", \"us_per_exchange\": %.3f, \"exchanges\": %u, "
           "\"gpu_polls_per_exchange\": %.2f}\n",
           dt * 1e6 / (N - 1), N - 1, r[0] ? double(r[1]) / r[0] : 0.0);
    fflush(stdout);
  }
  // 5. host write to fine-grained device memory (SIGSEGV caught and reported)
  {
    struct sigaction sa = {}, old = {};
    sa.sa_handler = on_segv;
    sigaction(SIGSEGV, &sa, &old);
    sigaction(SIGBUS, &sa, nullptr);
    int ok = -1;
    double us = 0;
    if (sigsetjmp(g_jb, 1) == 0) {
      volatile uint32_t* f = fg;
      f[0] = 0x12345678u;
      ok = f[0] == 0x12345678u;
      // write bandwidth/latency of 4 KiB + flag from the host (write-combined?)
      const double t0 = now_s();
      for (int rep = 0; rep < 1000; ++rep) {
        for (int i = 0; i < 1024; ++i) f[64 + i] = rep + i;
        __builtin_ia32_sfence();
      }
      us = (now_s() - t0) * 1e3;
    }
    sigaction(SIGSEGV, &old, nullptr);
    printf("{\"probe\": \"host_write_finegrained_device\", \"ok\": %d, \"us_per_4KiB_write\": %.3f}\n", ok, us);
  }
  return 0;
}
