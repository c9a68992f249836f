// gpu_stress — the supervised workload for the GPU-attribution scenarios
// (BASELINE.json config 3: "supervise 8 ROCm stress pods (one per GPU), inject
// HBM-OOM").  It is a test workload the supervisor *watches*, not part of the
// supervisor (which runs no GPU compute).  The reference has no equivalent.
//
//   gpu_stress hold    --gib G --seconds S     allocate G GiB, run an FMA loop for S s, exit 0
//   gpu_stress hbm-oom --chunk-gib C [--linger S] [--termination-log PATH]
//        allocate + touch C-GiB chunks until hipMalloc reports hipErrorOutOfMemory,
//        hold the peak for S s (so the node monitor samples it), write the HIP error
//        to PATH (the pod's terminationMessagePath) and exit 1.
//   gpu_stress hbm-oom --chunk-gib C --no-termination-log --linger 0
//        what a default PyTorch pod does: the OOM goes to stderr only, in torch's own
//        "torch.OutOfMemoryError: HIP out of memory. Tried to allocate … GPU N has a
//        total capacity of …" wording, and the process exits 1 at once (its VRAM is
//        freed by the exit, nothing lingers for a sampler to see).
//
// Kernels are sized for CDNA4: 256-thread workgroups (4 × 64-wide wavefronts),
// grid = 8 workgroups per CU over the 256 CUs, grid-stride loops, 16-byte stores.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CHECK(x)                                                                             \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "%s failed: %s (%s)\n", #x, hipGetErrorName(e_), hipGetErrorString(e_)); \
      exit(3);                                                                               \
    }                                                                                        \
  } while (0)

__global__ __launch_bounds__(256) void fill_kernel(uint4* __restrict__ p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (; i < n; i += stride) {
    uint32_t v = seed ^ static_cast<uint32_t>(i);
    p[i] = make_uint4(v, v + 1, v + 2, v + 3);
  }
}

__global__ __launch_bounds__(256) void fma_kernel(float* __restrict__ out, size_t n, int iters) {
  size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (; i < n; i += stride) {
    float a = out[i], b = 1.0001f, c = 0.9999f;
#pragma unroll 8
    for (int k = 0; k < iters; ++k) a = fmaf(a, b, c);
    out[i] = a;
  }
}

static const char* env_or(const char* k, const char* d) {
  const char* v = getenv(k);
  return v ? v : d;
}

static int grid_for(int dev) {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, dev));
  return prop.multiProcessorCount * 8;
}

static void write_termination(const std::string& path, const std::string& msg) {
  if (path.empty()) return;
  FILE* f = fopen(path.c_str(), "w");
  if (!f) return;
  fputs(msg.c_str(), f);
  fclose(f);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: gpu_stress hold|hbm-oom [--gib G] [--seconds S] [--chunk-gib C] [--linger S] "
                    "[--termination-log PATH | --no-termination-log] [--max-gib M] [--device D]\n");
    return 2;
  }
  std::string mode = argv[1];
  double gib = 1.0, seconds = 2.0, chunk_gib = 32.0, linger = 1.0, max_gib = 1e9;
  int device = 0;
  std::string term_log;
  bool no_term_log = false;
  for (int i = 2; i < argc;) {
    std::string k = argv[i];
    if (k == "--no-termination-log") {
      no_term_log = true;
      i += 1;
      continue;
    }
    if (i + 1 >= argc) {
      fprintf(stderr, "option %s needs a value\n", k.c_str());
      return 2;
    }
    const char* v = argv[i + 1];
    i += 2;
    if (k == "--gib") gib = atof(v);
    else if (k == "--seconds") seconds = atof(v);
    else if (k == "--chunk-gib") chunk_gib = atof(v);
    else if (k == "--linger") linger = atof(v);
    else if (k == "--max-gib") max_gib = atof(v);
    else if (k == "--device") device = atoi(v);
    else if (k == "--termination-log") term_log = v;
    else {
      fprintf(stderr, "unknown option %s\n", k.c_str());
      return 2;
    }
  }
  if (no_term_log) term_log.clear();
  CHECK(hipSetDevice(device));
  const int grid = grid_for(device);
  printf("gpu_stress %s device=%d rank=%s local_rank=%s world=%s visible=%s\n", mode.c_str(), device,
         env_or("RANK", "-"), env_or("LOCAL_RANK", "-"), env_or("WORLD_SIZE", "-"), env_or("HIP_VISIBLE_DEVICES", "-"));
  fflush(stdout);

  if (mode == "hold") {
    size_t bytes = static_cast<size_t>(gib * (1ull << 30)) & ~static_cast<size_t>(15);
    if (bytes < 16) bytes = 16;
    void* p = nullptr;
    CHECK(hipMalloc(&p, bytes));
    hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), 0, 0, static_cast<uint4*>(p), bytes / 16, 7u);
    CHECK(hipGetLastError());
    auto t0 = std::chrono::steady_clock::now();
    int rounds = 0;
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
      // the whole allocation is filled once (resident); the busy loop runs over its first
      // GiB only, so a multi-hundred-GiB hold still checks the clock every few ms
      hipLaunchKernelGGL(fma_kernel, dim3(grid), dim3(256), 0, 0, static_cast<float*>(p),
                         std::min(bytes / 4, static_cast<size_t>(1) << 28), 256);
      CHECK(hipGetLastError());
      CHECK(hipDeviceSynchronize());
      ++rounds;
    }
    printf("hold done: %.2f GiB, %d rounds\n", bytes / double(1ull << 30), rounds);
    CHECK(hipFree(p));
    return 0;
  }

  if (mode == "hbm-oom") {
    std::vector<void*> chunks;
    size_t chunk = static_cast<size_t>(chunk_gib * (1ull << 30)) & ~static_cast<size_t>(15);
    size_t total = 0;
    size_t free_b = 0, total_b = 0;
    CHECK(hipMemGetInfo(&free_b, &total_b));
    while (true) {
      if (total / double(1ull << 30) >= max_gib) {
        fprintf(stderr, "reached --max-gib %.1f without OOM\n", max_gib);
        return 4;
      }
      void* p = nullptr;
      hipError_t e = hipMalloc(&p, chunk);
      if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
        (void)hipGetLastError();  // clear the sticky-free error state
        char msg[768];
        size_t free_now = 0, total_now = 0;
        (void)hipMemGetInfo(&free_now, &total_now);
        if (no_term_log) {
          // torch's caching-allocator wording (what a default pod leaves in its log only)
          snprintf(msg, sizeof msg,
                   "torch.OutOfMemoryError: HIP out of memory. Tried to allocate %.2f GiB. GPU %d has a total "
                   "capacity of %.2f GiB of which %.2f GiB is free. Of the allocated memory %.2f GiB is allocated "
                   "by PyTorch, and 0 bytes is reserved by PyTorch but unallocated.",
                   chunk / double(1ull << 30), device, total_b / double(1ull << 30), free_now / double(1ull << 30),
                   total / double(1ull << 30));
          fprintf(stderr, "Traceback (most recent call last):\n  File \"train.py\", line 42, in <module>\n%s\n", msg);
        } else {
          snprintf(msg, sizeof msg,
                   "%s: HIP out of memory. Tried to allocate %.2f GiB. GPU %d has a total capacity of %.2f GiB; "
                   "%.2f GiB already allocated by this process (rank=%s local_rank=%s)",
                   hipGetErrorName(e), chunk / double(1ull << 30), device, total_b / double(1ull << 30),
                   total / double(1ull << 30), env_or("RANK", "-"), env_or("LOCAL_RANK", "-"));
          fprintf(stderr, "%s\n", msg);
        }
        fflush(stderr);
        write_termination(term_log, msg);
        if (linger > 0) std::this_thread::sleep_for(std::chrono::duration<double>(linger));
        for (void* q : chunks) (void)hipFree(q);
        return 1;
      }
      CHECK(e);
      hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), 0, 0, static_cast<uint4*>(p), chunk / 16,
                         static_cast<uint32_t>(chunks.size()));
      CHECK(hipGetLastError());
      CHECK(hipDeviceSynchronize());
      chunks.push_back(p);
      total += chunk;
      printf("allocated %.1f GiB\n", total / double(1ull << 30));
      fflush(stdout);
    }
  }
  fprintf(stderr, "unknown mode %s\n", mode.c_str());
  return 2;
}
