// rccl-allreduce-bench — RCCL all-reduce bandwidth + correctness over xGMI, one pod × N GPUs.
//
// BASELINE.json config 4 ("Pod requesting amd.com/gpu:8 runs RCCL all-reduce bandwidth test over
// xGMI"); the reference leaves the multi-GPU-pod case as "TBD" (reference README.md:389-391) and
// has no collective call sites at all.  Single process drives every GPU the device
// plugin allocated (ncclCommInitAll + group calls), nccl-tests style:
//
//   size  count  type  time(us)  algbw(GB/s)  busbw(GB/s)  #wrong
//
// With --mp it runs as ONE RANK of a one-process-per-GPU job instead — the topology bench.py and
// every torch.distributed job use — launched as
//   torchrun --nproc-per-node N --no-python rccl-allreduce-bench --mp [...]
// (RANK / WORLD_SIZE / LOCAL_RANK from the launcher; rank 0 publishes the ncclUniqueId through a file
// that the other ranks poll, then ncclCommInitRank); times are the MAX over ranks and rank 0 prints.
// --plan prints the resolved launch (mode, rank, world, device, id file) and exits before any HIP call.
//
// The id file is keyed per launch, never just per port: <run id>.<launcher pid>.<restart>.<port>.
// Every rank of one torchrun launch shares its parent (the elastic agent), whose pid is unique among
// live processes; the Job also sets --rdzv-id to the pod UID.  A reader only accepts a file written
// after the launcher started (mtime >= the agent's start time from /proc), so a stale file left in a
// reused /tmp by a crashed earlier launch is ignored (rank 0 also removes it before publishing).
//
// busbw = algbw · 2(n−1)/n (ring all-reduce traffic per rank).  On MI355X each GPU has 7 xGMI links
// of ~153 GB/s; a ring uses one outgoing link per hop, so RCCL reaches beyond one link only by
// spreading channels over several rings — report what is measured, not the aggregate link rate.
// Correctness: rank r contributes (r+1) in every element; after the sum every element must be
// n(n+1)/2 (exact in bf16 for n ≤ 8 and in fp32 always).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "amdk8s_native.h"

#define RCCL_CHECK(expr)                                                                       \
  do {                                                                                         \
    ncclResult_t _r = (expr);                                                                  \
    if (_r != ncclSuccess) {                                                                   \
      std::fprintf(stderr, "RCCL error %s at %s:%d: %s\n", ncclGetErrorString(_r), __FILE__,   \
                   __LINE__, #expr);                                                           \
      std::exit(3);                                                                            \
    }                                                                                          \
  } while (0)

namespace {

__global__ void fill_f32(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

__global__ void count_wrong_f32(const float* p, size_t n, float expect, unsigned long long* bad) {
  unsigned long long local = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    local += (p[i] != expect);
  if (local) atomicAdd(bad, local);
}

struct Options {
  size_t min_bytes = 8;
  size_t max_bytes = (size_t)1 << 30;
  int factor = 4;
  int iters = 20;
  int warmup = 5;
  int ngpus = 0;  // 0 = all visible
  bool json = false;
  bool mp = false;    // one rank of a one-process-per-GPU job
  bool plan = false;  // print the resolved launch and exit
  std::string id_file;
  int id_timeout_s = 300;
};

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

// Wall-clock start time (s since the epoch) of process `pid`: /proc/<pid>/stat field 22 (clock
// ticks after boot) + btime of /proc/stat.  -1 when unreadable.
double process_start_time(pid_t pid) {
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
  FILE* f = std::fopen(path, "r");
  if (!f) return -1;
  char buf[4096];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* p = std::strrchr(buf, ')');   // comm may contain spaces
  if (!p) return -1;
  unsigned long long start = 0;
  int field = 2;
  for (const char* q = p + 1; *q && field < 22; ++q)
    if (*q == ' ' && ++field == 22) start = std::strtoull(q + 1, nullptr, 10);
  FILE* st = std::fopen("/proc/stat", "r");
  if (!st) return -1;
  char line[256];
  double btime = -1;
  while (std::fgets(line, sizeof(line), st))
    if (std::strncmp(line, "btime ", 6) == 0) btime = std::strtod(line + 6, nullptr);
  std::fclose(st);
  if (btime < 0 || start == 0) return -1;
  return btime + (double)start / (double)sysconf(_SC_CLK_TCK);
}

// Launch key shared by every rank of one torchrun launch (see the header comment).
std::string launch_key() {
  const char* run = std::getenv("TORCHELASTIC_RUN_ID");
  const char* restart = std::getenv("TORCHELASTIC_RESTART_COUNT");
  const char* port = std::getenv("MASTER_PORT");
  return std::string(run && *run ? run : "none") + "." + std::to_string((long)getppid()) + "." +
         (restart && *restart ? restart : "0") + "." + (port ? port : "0");
}

// A file at `path` that this launch may read: written no earlier than the launcher's start
// (1 s slack for mtime granularity).  Without /proc the check is skipped (fresh = true).
bool id_file_fresh(const std::string& path, double not_before) {
  struct stat sb;
  if (stat(path.c_str(), &sb) != 0) return false;
  if (not_before < 0) return true;
  const double mtime = (double)sb.st_mtim.tv_sec + 1e-9 * (double)sb.st_mtim.tv_nsec;
  return mtime >= not_before - 1.0;
}

// rank 0 → file (stale copy removed first, then atomic rename); others poll for a FRESH file
bool exchange_id(ncclUniqueId* id, int rank, const std::string& path, int timeout_s,
                 double not_before) {
  if (rank == 0) {
    std::remove(path.c_str());
    const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f || std::fwrite(id, sizeof(*id), 1, f) != 1) return false;
    std::fclose(f);
    return std::rename(tmp.c_str(), path.c_str()) == 0;
  }
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
  while (std::chrono::steady_clock::now() < deadline) {
    if (id_file_fresh(path, not_before)) {
      FILE* f = std::fopen(path.c_str(), "rb");
      if (f) {
        const bool ok = std::fread(id, sizeof(*id), 1, f) == 1;
        std::fclose(f);
        if (ok) return true;
      }
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  return false;
}

size_t parse_size(const char* s) {
  char* end = nullptr;
  double v = std::strtod(s, &end);
  std::string suf = end ? end : "";
  if (suf == "K" || suf == "k") v *= 1024;
  else if (suf == "M" || suf == "m") v *= 1024 * 1024;
  else if (suf == "G" || suf == "g") v *= 1024.0 * 1024 * 1024;
  return (size_t)v;
}

int run_mp(const Options& o, int rank, int world, int local) {
  AMDK8S_HIP_CHECK(hipSetDevice(local));
  ncclUniqueId id;
  if (rank == 0) RCCL_CHECK(ncclGetUniqueId(&id));
  if (!exchange_id(&id, rank, o.id_file, o.id_timeout_s, process_start_time(getppid()))) {
    std::fprintf(stderr, "rank %d: no ncclUniqueId at %s after %d s\n", rank, o.id_file.c_str(),
                 o.id_timeout_s);
    return 3;
  }
  ncclComm_t comm;
  RCCL_CHECK(ncclCommInitRank(&comm, world, id, rank));
  if (rank == 0) std::remove(o.id_file.c_str());   // every rank has read it by now
  int ver = 0;
  ncclGetVersion(&ver);
  hipStream_t st;
  AMDK8S_HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const size_t max_count = std::max<size_t>(1, o.max_bytes / sizeof(float));
  float* buf = nullptr;
  double* scal = nullptr;   // [0] time (max over ranks), [1] wrong count (sum)
  unsigned long long* dbad = nullptr;
  AMDK8S_HIP_CHECK(hipMalloc(&buf, max_count * sizeof(float)));
  AMDK8S_HIP_CHECK(hipMalloc(&scal, 2 * sizeof(double)));
  AMDK8S_HIP_CHECK(hipMalloc(&dbad, sizeof(unsigned long long)));
  if (rank == 0) {
    std::printf("# rccl-allreduce-bench --mp: %d rank(s), one GPU each, RCCL %d, in-place float "
                "sum, %d iters\n", world, ver, o.iters);
    std::printf("# %12s %12s %6s %10s %12s %12s %8s\n", "size(B)", "count", "type", "time(us)",
                "algbw(GB/s)", "busbw(GB/s)", "#wrong");
  }
  auto barrier = [&]() {
    RCCL_CHECK(ncclAllReduce(scal, scal, 1, ncclFloat64, ncclMax, comm, st));
    AMDK8S_HIP_CHECK(hipStreamSynchronize(st));
  };
  double peak_bus = 0, peak_alg = 0;
  size_t peak_size = 0;
  unsigned long long total_bad = 0;
  const float expect = (float)world * (world + 1) / 2.0f;
  for (size_t bytes = o.min_bytes; bytes <= o.max_bytes; bytes *= (size_t)o.factor) {
    const size_t count = std::max<size_t>(1, bytes / sizeof(float));
    hipLaunchKernelGGL(fill_f32, dim3(1024), dim3(256), 0, st, buf, count, (float)(rank + 1));
    AMDK8S_HIP_CHECK(hipMemsetAsync(dbad, 0, sizeof(unsigned long long), st));
    RCCL_CHECK(ncclAllReduce(buf, buf, count, ncclFloat, ncclSum, comm, st));
    hipLaunchKernelGGL(count_wrong_f32, dim3(1024), dim3(256), 0, st, buf, count, expect, dbad);
    unsigned long long b = 0;
    AMDK8S_HIP_CHECK(hipMemcpyAsync(&b, dbad, sizeof(b), hipMemcpyDeviceToHost, st));
    AMDK8S_HIP_CHECK(hipStreamSynchronize(st));
    for (int w = 0; w < o.warmup; ++w)
      RCCL_CHECK(ncclAllReduce(buf, buf, count, ncclFloat, ncclSum, comm, st));
    barrier();
    auto t0 = std::chrono::steady_clock::now();
    for (int it = 0; it < o.iters; ++it)
      RCCL_CHECK(ncclAllReduce(buf, buf, count, ncclFloat, ncclSum, comm, st));
    AMDK8S_HIP_CHECK(hipStreamSynchronize(st));
    double h[2] = {std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                       .count() / o.iters, (double)b};
    AMDK8S_HIP_CHECK(hipMemcpyAsync(scal, h, sizeof(h), hipMemcpyHostToDevice, st));
    RCCL_CHECK(ncclAllReduce(scal, scal, 1, ncclFloat64, ncclMax, comm, st));
    RCCL_CHECK(ncclAllReduce(scal + 1, scal + 1, 1, ncclFloat64, ncclSum, comm, st));
    AMDK8S_HIP_CHECK(hipMemcpyAsync(h, scal, sizeof(h), hipMemcpyDeviceToHost, st));
    AMDK8S_HIP_CHECK(hipStreamSynchronize(st));
    const double us = h[0];
    const unsigned long long bad = (unsigned long long)h[1];
    total_bad += bad;
    const double algbw = (double)count * sizeof(float) / (us * 1e-6) / 1e9;
    const double busbw = world > 1 ? algbw * 2.0 * (world - 1) / world : algbw;
    if (busbw > peak_bus) {
      peak_bus = busbw;
      peak_alg = algbw;
      peak_size = count * sizeof(float);
    }
    if (rank == 0)
      std::printf("  %12zu %12zu %6s %10.1f %12.2f %12.2f %8llu\n", count * sizeof(float), count,
                  "float", us, algbw, busbw, bad);
    if (bytes > o.max_bytes / (size_t)o.factor) break;
  }
  if (rank == 0) {
    std::printf("# peak busbw %.2f GB/s (algbw %.2f GB/s) at %zu bytes on %d rank(s)\n", peak_bus,
                peak_alg, peak_size, world);
    if (o.json)
      std::printf("{\"check\": \"rccl_allreduce\", \"mode\": \"mp\", \"ngpus\": %d, "
                  "\"peak_busbw_gbps\": %.2f, \"peak_algbw_gbps\": %.2f, \"peak_bytes\": %zu, "
                  "\"wrong\": %llu, \"passed\": %s}\n", world, peak_bus, peak_alg, peak_size, total_bad,
                  total_bad == 0 ? "true" : "false");
    std::printf(total_bad ? "Test FAILED\n" : "Test PASSED\nDone\n");
  }
  ncclCommDestroy(comm);
  hipFree(buf);
  hipFree(scal);
  hipFree(dbad);
  hipStreamDestroy(st);
  return total_bad ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
      return argv[++i];
    };
    if (a == "-b" || a == "--minbytes") o.min_bytes = parse_size(next());
    else if (a == "-e" || a == "--maxbytes") o.max_bytes = parse_size(next());
    else if (a == "-f" || a == "--stepfactor") o.factor = std::atoi(next());
    else if (a == "-n" || a == "--iters") o.iters = std::atoi(next());
    else if (a == "-w" || a == "--warmup") o.warmup = std::atoi(next());
    else if (a == "-g" || a == "--ngpus") o.ngpus = std::atoi(next());
    else if (a == "--json") o.json = true;
    else if (a == "--mp") o.mp = true;
    else if (a == "--plan") o.plan = true;
    else if (a == "--id-file") o.id_file = next();
    else if (a == "--id-timeout") o.id_timeout_s = std::atoi(next());
    else {
      std::printf("usage: rccl-allreduce-bench [-b MIN] [-e MAX] [-f FACTOR] [-n ITERS] "
                  "[-w WARMUP] [-g NGPUS] [--json] [--mp [--id-file PATH] [--id-timeout S]] "
                  "[--plan]\n");
      return a == "-h" || a == "--help" ? 0 : 2;
    }
  }
  if (o.mp) {
    const int rank = env_int("RANK", -1), world = env_int("WORLD_SIZE", -1);
    const int local = env_int("LOCAL_RANK", rank);
    if (rank < 0 || world < 1 || rank >= world) {
      std::fprintf(stderr, "--mp needs RANK and WORLD_SIZE (launch with torchrun --no-python)\n");
      return 2;
    }
    if (o.id_file.empty()) {
      const char* tmpdir = std::getenv("TMPDIR");
      o.id_file = std::string(tmpdir && *tmpdir ? tmpdir : "/tmp") + "/rccl-allreduce-bench." +
                  launch_key() + ".id";
    }
    if (o.plan) {
      const double not_before = process_start_time(getppid());
      std::printf("{\"mode\": \"mp\", \"rank\": %d, \"world\": %d, \"device\": %d, "
                  "\"id_file\": \"%s\", \"launcher_start\": %.3f, \"existing_id_file_fresh\": %s}\n",
                  rank, world, local, o.id_file.c_str(), not_before,
                  id_file_fresh(o.id_file, not_before) ? "true" : "false");
      return 0;
    }
    return run_mp(o, rank, world, local);
  }
  if (o.plan) {
    std::printf("{\"mode\": \"single\", \"ngpus\": %d}\n", o.ngpus);
    return 0;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    std::fprintf(stderr, "No HIP device visible to this container\n");
    return 1;
  }
  const int n = o.ngpus > 0 ? std::min(o.ngpus, ndev) : ndev;
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(n);
  RCCL_CHECK(ncclCommInitAll(comms.data(), n, devs.data()));
  int ver = 0;
  ncclGetVersion(&ver);

  std::vector<float*> buf(n);
  std::vector<hipStream_t> st(n);
  std::vector<unsigned long long*> dbad(n);
  const size_t max_count = std::max<size_t>(1, o.max_bytes / sizeof(float));
  for (int i = 0; i < n; ++i) {
    AMDK8S_HIP_CHECK(hipSetDevice(devs[i]));
    AMDK8S_HIP_CHECK(hipMalloc(&buf[i], max_count * sizeof(float)));
    AMDK8S_HIP_CHECK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    AMDK8S_HIP_CHECK(hipMalloc(&dbad[i], sizeof(unsigned long long)));
  }
  std::printf("# rccl-allreduce-bench: %d GPU(s), RCCL %d, in-place float sum, %d iters\n", n, ver,
              o.iters);
  std::printf("# %12s %12s %6s %10s %12s %12s %8s\n", "size(B)", "count", "type", "time(us)",
              "algbw(GB/s)", "busbw(GB/s)", "#wrong");
  double peak_bus = 0, peak_alg = 0;
  size_t peak_size = 0;
  unsigned long long total_bad = 0;
  const float expect = (float)n * (n + 1) / 2.0f;
  for (size_t bytes = o.min_bytes; bytes <= o.max_bytes; bytes *= (size_t)o.factor) {
    const size_t count = std::max<size_t>(1, bytes / sizeof(float));
    // correctness pass
    for (int i = 0; i < n; ++i) {
      AMDK8S_HIP_CHECK(hipSetDevice(devs[i]));
      hipLaunchKernelGGL(fill_f32, dim3(1024), dim3(256), 0, st[i], buf[i], count, (float)(i + 1));
      AMDK8S_HIP_CHECK(hipMemsetAsync(dbad[i], 0, sizeof(unsigned long long), st[i]));
    }
    RCCL_CHECK(ncclGroupStart());
    for (int i = 0; i < n; ++i)
      RCCL_CHECK(ncclAllReduce(buf[i], buf[i], count, ncclFloat, ncclSum, comms[i], st[i]));
    RCCL_CHECK(ncclGroupEnd());
    unsigned long long bad = 0;
    for (int i = 0; i < n; ++i) {
      AMDK8S_HIP_CHECK(hipSetDevice(devs[i]));
      hipLaunchKernelGGL(count_wrong_f32, dim3(1024), dim3(256), 0, st[i], buf[i], count, expect,
                         dbad[i]);
      unsigned long long b = 0;
      AMDK8S_HIP_CHECK(hipMemcpyAsync(&b, dbad[i], sizeof(b), hipMemcpyDeviceToHost, st[i]));
      AMDK8S_HIP_CHECK(hipStreamSynchronize(st[i]));
      bad += b;
    }
    total_bad += bad;
    // timed passes (values grow; only bandwidth matters here)
    auto launch = [&]() {
      RCCL_CHECK(ncclGroupStart());
      for (int i = 0; i < n; ++i)
        RCCL_CHECK(ncclAllReduce(buf[i], buf[i], count, ncclFloat, ncclSum, comms[i], st[i]));
      RCCL_CHECK(ncclGroupEnd());
    };
    for (int w = 0; w < o.warmup; ++w) launch();
    for (int i = 0; i < n; ++i) {
      AMDK8S_HIP_CHECK(hipSetDevice(devs[i]));
      AMDK8S_HIP_CHECK(hipStreamSynchronize(st[i]));
    }
    auto t0 = std::chrono::steady_clock::now();
    for (int it = 0; it < o.iters; ++it) launch();
    for (int i = 0; i < n; ++i) {
      AMDK8S_HIP_CHECK(hipSetDevice(devs[i]));
      AMDK8S_HIP_CHECK(hipStreamSynchronize(st[i]));
    }
    const double us =
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() /
        o.iters;
    const double algbw = (double)count * sizeof(float) / (us * 1e-6) / 1e9;
    const double busbw = n > 1 ? algbw * 2.0 * (n - 1) / n : algbw;
    if (busbw > peak_bus) {
      peak_bus = busbw;
      peak_alg = algbw;
      peak_size = count * sizeof(float);
    }
    std::printf("  %12zu %12zu %6s %10.1f %12.2f %12.2f %8llu\n", count * sizeof(float), count,
                "float", us, algbw, busbw, bad);
    if (bytes > o.max_bytes / (size_t)o.factor) break;
  }
  std::printf("# peak busbw %.2f GB/s (algbw %.2f GB/s) at %zu bytes on %d GPU(s)\n", peak_bus,
              peak_alg, peak_size, n);
  if (o.json)
    std::printf("{\"check\": \"rccl_allreduce\", \"ngpus\": %d, \"peak_busbw_gbps\": %.2f, "
                "\"peak_algbw_gbps\": %.2f, \"peak_bytes\": %zu, \"wrong\": %llu, \"passed\": %s}\n",
                n, peak_bus, peak_alg, peak_size, total_bad, total_bad == 0 ? "true" : "false");
  for (int i = 0; i < n; ++i) {
    ncclCommDestroy(comms[i]);
    hipFree(buf[i]);
    hipFree(dbad[i]);
    hipStreamDestroy(st[i]);
  }
  if (total_bad) {
    std::printf("Test FAILED\n");
    return 1;
  }
  std::printf("Test PASSED\nDone\n");
  return 0;
}
