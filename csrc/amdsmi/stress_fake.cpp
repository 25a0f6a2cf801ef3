// Concurrency + memory-safety driver for libnos_amdsmi's fake backend
// (the C++ library gets ThreadSanitizer and
// AddressSanitizer/UBSan builds).  Compiled together with nos_amdsmi.cpp by
// tests/test_native_sanitizers.py with -fsanitize=thread or
// -fsanitize=address,undefined; the sanitizer runtime aborts on any report.
//
// Readers (gpu_info / activity / processes / link) race writers (partition
// switches, process add/remove, fault injection) from 8 threads.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

struct nos_gpu_info {
  int index, num_cus, num_xcds, compute_mode, memory_mode, num_partitions, hip_id, drm_render;
  long long vram_mb;
  char bdf[32];
  char uuid[64];
  char market_name[128];
};
struct nos_proc_info {
  unsigned pid, cu_occupancy;
  long long vram_bytes;
  char name[64];
};

extern "C" {
int nos_smi_open(const char* backend, const char* spec, int allow_set);
int nos_smi_close();
int nos_smi_count();
int nos_smi_gpu_info(int i, nos_gpu_info* out);
int nos_smi_set_compute_partition(int i, int mode);
int nos_smi_set_memory_partition(int i, int mode);
int nos_smi_activity(int i, int* gfx, int* umc, int* mm);
int nos_smi_processes(int i, nos_proc_info* out, int max, int* n);
int nos_smi_link(int i, int j, int* type, long long* hops, long long* weight);
int nos_smi_fake_inject(const char* fault);
int nos_smi_fake_add_process(int i, unsigned pid, long long vram, unsigned cus);
int nos_smi_fake_remove_process(int i, unsigned pid);
int nos_smi_fake_set_activity(int i, int gfx, int umc);
int nos_smi_struct_sizes(int* gpu_info, int* proc_info);
int nos_smi_rescan();
}

int main() {
  int a = 0, b = 0;
  nos_smi_struct_sizes(&a, &b);
  if (a != (int)sizeof(nos_gpu_info) || b != (int)sizeof(nos_proc_info)) {
    std::fprintf(stderr, "ABI mismatch %d/%zu %d/%zu\n", a, sizeof(nos_gpu_info), b, sizeof(nos_proc_info));
    return 2;
  }
  if (nos_smi_open("fake", "gpus=8;cus=256;xcds=8;vram_mb=294912;compute=SPX;memory=NPS1", 1) != 0) return 3;
  const int n = nos_smi_count();
  if (n != 8) return 4;
  std::atomic<long> ops{0};
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t) {
    th.emplace_back([&, t] {
      for (int it = 0; it < 2000; ++it) {
        const int g = (t + it) % n;
        nos_gpu_info info;
        std::memset(&info, 0, sizeof(info));
        if (nos_smi_gpu_info(g, &info) == 0 && (info.num_partitions < 1 || info.num_partitions > 8)) ++bad;
        if (t % 4 == 0) {
          static const int modes[] = {1, 2, 4, 5};
          nos_smi_set_compute_partition(g, modes[it % 4]);  // may fail while "busy": fine
        } else if (t % 4 == 1) {
          nos_smi_fake_add_process(g, 1000 + t, 1 << 20, 8);
          nos_proc_info procs[16];
          int np = 0;
          nos_smi_processes(g, procs, 16, &np);
          if (np < 0 || np > 16) ++bad;
          nos_smi_fake_remove_process(g, 1000 + t);
        } else if (t % 4 == 2) {
          int gfx, umc, mm;
          nos_smi_fake_set_activity(g, it % 100, it % 50);
          nos_smi_activity(g, &gfx, &umc, &mm);
          int type;
          long long hops, w;
          nos_smi_link(g, (g + 1) % n, &type, &hops, &w);
        } else {
          nos_smi_fake_inject(it % 2 ? "fail_set_compute" : "clear");
          nos_smi_set_memory_partition(g, it % 2 ? 2 : 1);
          // another process switches a mode; this session re-enumerates (deferred
          // while one of its own switches -- run outside the lock -- is in flight)
          nos_smi_fake_inject(it % 3 ? "external_switch=3:CPX" : "external_switch=3:SPX");
          if (it % 50 == 0) nos_smi_fake_inject("switch_delay_ms=1");
          nos_smi_rescan();
        }
        ++ops;
      }
    });
  }
  for (auto& x : th) x.join();
  nos_smi_fake_inject("clear");
  nos_smi_close();
  std::printf("ops=%ld bad=%d\n", ops.load(), bad.load());
  return bad.load() == 0 ? 0 : 1;
}
