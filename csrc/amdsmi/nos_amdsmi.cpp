// libnos_amdsmi — the node-local device access layer of the nos-amd agents.
//
// Replaces the reference's cgo NVML client (pkg/gpu/nvml/client.go:37-518,
// interface pkg/gpu/nvml/interface.go:23-35) with an amd-smi based one:
// instead of creating/destroying MIG GPU/compute instances it reads and sets
// the GPU-wide compute partition (SPX/DPX/QPX/CPX) and memory partition
// (NPS1/NPS4), lists the logical devices a partition mode exposes, the
// processes on a GPU (drain check before a repartition), engine activity and
// the xGMI topology.
//
// Two backends behind one C ABI (loaded from Python with ctypes):
//   * "amdsmi": dlopen()s libamd_smi.so at open time (no link-time
//     dependency, so the library loads on machines without ROCm);
//   * "fake":   an in-memory MI355X node with programmable partitions,
//     processes, activity and fault injection, used by the simulator and tests
//     (the role of the reference's hand-written mocks/mig.Client,
//     pkg/test/mocks/mig/mig_client.go:27-80).
//
// Physical GPUs vs logical partitions: in DPX/QPX/CPX amd-smi enumerates one
// processor handle PER PARTITION.  The library groups those handles back into
// physical GPUs (by amd-smi socket, i.e. the device's PCI bus/device; the
// partitions of one socket ordered by their KFD partition id) -- the role of
// the reference's GetMigDeviceGpuIndex / parent-GPU lookup
// (pkg/gpu/nvml/client.go:59-146).  nos_smi_count()/gpu_info() report
// physical GPUs (the unit of a mode switch and of the node's GPU count);
// nos_smi_partition_count()/partition_info() report the logical devices of
// one GPU with their own HIP id, render node, CUs, XCDs and memory.
//
// All entry points are serialised by one mutex (the reference's NVML client
// does Init/Shutdown per call, client.go:46-57; we keep one session open) --
// except the slow part of a mode switch: nos_smi_set_*_partition validate and
// mark the GPU "switching" under the mutex, call the driver WITHOUT it, then
// re-enumerate under it again.  Queries about other GPUs keep answering while
// a switch runs (or hangs); queries about the switching GPU return
// NOS_SMI_ERR_SWITCHING instead of blocking.  The partition agent bounds the
// switch with its own deadline (agents/partagent.py).
//
// The session enumerates handles at open time and after its own switches,
// like amd-smi: a mode changed by ANOTHER process (another agent, amd-smi CLI)
// is invisible until nos_smi_rescan() -- the device plugin calls it on every
// poll.  The fake backend models that with a separate "hardware" state and
// session view (fault "external_switch=<gpu>:<mode>").
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <amd_smi/amdsmi.h>

#define NOS_API extern "C" __attribute__((visibility("default")))

enum NosSmiError : int {
  NOS_SMI_OK = 0,
  NOS_SMI_ERR_NOT_OPEN = -1,
  NOS_SMI_ERR_BAD_INDEX = -2,
  NOS_SMI_ERR_BACKEND = -3,
  NOS_SMI_ERR_UNSUPPORTED = -4,
  NOS_SMI_ERR_BUSY = -5,        // processes still on the GPU
  NOS_SMI_ERR_INJECTED = -6,    // fake backend fault injection
  NOS_SMI_ERR_INVALID = -7,
  NOS_SMI_ERR_TIMEOUT = -8,
  NOS_SMI_ERR_SWITCHING = -9,   // a mode switch of this GPU is in progress
};

// compute modes: 1=SPX 2=DPX 3=TPX 4=QPX 5=CPX (amdsmi_compute_partition_type_t)
// memory modes: 1=NPS1 2=NPS2 4=NPS4 8=NPS8 (amdsmi_memory_partition_type_t)

struct nos_gpu_info {
  int index;
  int num_cus;
  int num_xcds;
  int compute_mode;
  int memory_mode;
  int num_partitions;  // logical devices the current compute mode exposes
  int hip_id;
  int drm_render;
  long long vram_mb;
  char bdf[32];
  char uuid[64];
  char market_name[128];
};

struct nos_part_info {
  int gpu_index;       // physical GPU
  int partition;       // index of the logical device within its GPU
  int hip_id;          // HIP device ordinal of the logical device
  int drm_render;      // /dev/dri/renderD<n>
  int kfd_node;
  int num_cus;
  int num_xcds;
  int memory_shared;   // 1: partitions share one memory pool (NPS1), vram_mb is a fair share
  long long vram_mb;
  char bdf[32];
  char uuid[64];
};

struct nos_proc_info {
  unsigned pid;
  unsigned cu_occupancy;
  long long vram_bytes;
  char name[64];
};

namespace {

int partitions_for_mode(int mode) {
  switch (mode) {
    case 1: return 1;
    case 2: return 2;
    case 3: return 3;
    case 4: return 4;
    case 5: return 8;
    default: return 1;
  }
}

int parse_compute(const char* s) {
  if (!s) return 0;
  std::string m(s);
  if (m.find("SPX") != std::string::npos) return 1;
  if (m.find("DPX") != std::string::npos) return 2;
  if (m.find("TPX") != std::string::npos) return 3;
  if (m.find("QPX") != std::string::npos) return 4;
  if (m.find("CPX") != std::string::npos) return 5;
  return 0;
}

int parse_memory(const char* s) {
  if (!s) return 0;
  std::string m(s);
  if (m.find("NPS1") != std::string::npos) return 1;
  if (m.find("NPS2") != std::string::npos) return 2;
  if (m.find("NPS4") != std::string::npos) return 4;
  if (m.find("NPS8") != std::string::npos) return 8;
  return 0;
}

struct Backend {
  virtual ~Backend() = default;
  virtual int count() = 0;
  virtual int info(int i, nos_gpu_info* out) = 0;
  virtual int set_compute(int i, int mode) = 0;
  virtual int set_memory(int i, int mode) = 0;
  virtual int activity(int i, int* gfx, int* umc, int* mm) = 0;
  virtual int processes(int i, nos_proc_info* out, int max, int* n) = 0;
  virtual int link(int i, int j, int* type, long long* hops, long long* weight) = 0;
  virtual int partition_count(int i) = 0;
  virtual int clock(int i, int* cur_mhz, int* max_mhz) = 0;
  virtual int partition_info(int i, int p, nos_part_info* out) = 0;
  // re-read the device set (another process may have switched a mode)
  virtual int rescan() = 0;
  // mode switch in three steps: prepare (global lock held: validate, mark the
  // GPU switching), run (no global lock: the slow driver call), finish (lock
  // held: apply / re-enumerate, clear the mark)
  virtual int switch_prepare(int i, bool compute, int mode) = 0;
  virtual int switch_run(int i, bool compute, int mode) = 0;
  virtual int switch_finish(int i, bool compute, int mode, int rc) = 0;
  std::vector<char> switching;  // per GPU
  bool is_switching(int i) const { return i >= 0 && i < (int)switching.size() && switching[i]; }
  virtual int inject(const char* /*fault*/) { return NOS_SMI_ERR_UNSUPPORTED; }
  virtual int add_process(int, unsigned, long long, unsigned) { return NOS_SMI_ERR_UNSUPPORTED; }
  virtual int remove_process(int, unsigned) { return NOS_SMI_ERR_UNSUPPORTED; }
  virtual int set_activity(int, int, int) { return NOS_SMI_ERR_UNSUPPORTED; }
};

// ---------------------------------------------------------------- fake ----
struct FakeGpu {
  int compute = 1, memory = 1;
  int cus = 256, xcds = 8;
  long long vram_mb = 294912;  // 288 GiB
  int gfx = 0, umc = 0;
  bool lost = false;
  std::map<unsigned, nos_proc_info> procs;
};

struct FakeBackend : Backend {
  // gpus: the hardware; view: what this session enumerated (compute / memory
  // mode, lost) -- equal except after an external switch, until rescan()
  std::vector<FakeGpu> gpus;
  std::vector<FakeGpu> view;
  std::string model = "AMD Instinct MI355X";
  bool fail_set_compute = false, fail_set_memory = false, stale_mode = false;
  bool lose_after_switch = false;
  int switch_delay_ms = 0;

  explicit FakeBackend(const std::string& spec) {
    int n = 8;
    FakeGpu proto;
    // spec: "gpus=8;cus=256;xcds=8;vram_mb=294912;compute=SPX;memory=NPS1;model=..."
    size_t pos = 0;
    while (pos < spec.size()) {
      size_t end = spec.find(';', pos);
      if (end == std::string::npos) end = spec.size();
      std::string kv = spec.substr(pos, end - pos);
      size_t eq = kv.find('=');
      if (eq != std::string::npos) {
        std::string k = kv.substr(0, eq), v = kv.substr(eq + 1);
        if (k == "gpus") n = std::stoi(v);
        else if (k == "cus") proto.cus = std::stoi(v);
        else if (k == "xcds") proto.xcds = std::stoi(v);
        else if (k == "vram_mb") proto.vram_mb = std::stoll(v);
        else if (k == "compute") proto.compute = parse_compute(v.c_str());
        else if (k == "memory") proto.memory = parse_memory(v.c_str());
        else if (k == "model") model = v;
        else if (k == "switch_delay_ms") switch_delay_ms = std::stoi(v);
      }
      pos = end + 1;
    }
    if (proto.compute == 0) proto.compute = 1;
    if (proto.memory == 0) proto.memory = 1;
    gpus.assign(n, proto);
    view = gpus;
    switching.assign(n, 0);
    pending_delay_ms.assign(n, 0);  // sized once: switch_run reads it without the lock
  }

  bool ok(int i) const { return i >= 0 && i < (int)view.size() && !view[i].lost && !gpus[i].lost; }
  // a query about GPU i: not lost, not in the middle of a mode switch
  int check(int i) const {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    return is_switching(i) ? NOS_SMI_ERR_SWITCHING : NOS_SMI_OK;
  }

  int count() override { return (int)view.size(); }

  int rescan() override {
    for (int i = 0; i < (int)gpus.size(); ++i)
      if (is_switching(i)) return NOS_SMI_ERR_SWITCHING;
    view = gpus;
    return NOS_SMI_OK;
  }

  int info(int i, nos_gpu_info* o) override {
    if (int rc = check(i)) return rc;
    const FakeGpu& g = view[i];
    std::memset(o, 0, sizeof(*o));
    o->index = i;
    o->num_cus = g.cus;
    o->num_xcds = g.xcds;
    o->compute_mode = g.compute;
    o->memory_mode = g.memory;
    o->num_partitions = partitions_for_mode(g.compute);
    int base = 0;  // a GPU's HIP id / render node are those of its first logical device
    for (int j = 0; j < i; ++j)
      if (!view[j].lost) base += partitions_for_mode(view[j].compute);
    o->hip_id = base;
    o->drm_render = 128 + base;
    o->vram_mb = g.vram_mb;
    std::snprintf(o->bdf, sizeof(o->bdf), "0000:%02x:00.0", 0x05 + 0x10 * i);
    std::snprintf(o->uuid, sizeof(o->uuid), "GPU-fake-mi355x-%04d", i);
    std::snprintf(o->market_name, sizeof(o->market_name), "%s", model.c_str());
    return NOS_SMI_OK;
  }

  std::vector<int> pending_delay_ms;

  int switch_prepare(int i, bool compute, int mode) override {
    if (compute ? (mode < 1 || mode > 5) : (mode != 1 && mode != 2 && mode != 4 && mode != 8))
      return NOS_SMI_ERR_INVALID;
    if (int rc = check(i)) return rc;
    if (compute ? fail_set_compute : fail_set_memory) return NOS_SMI_ERR_INJECTED;
    if (!gpus[i].procs.empty()) return NOS_SMI_ERR_BUSY;
    pending_delay_ms[i] = switch_delay_ms;
    switching[i] = 1;
    return NOS_SMI_OK;
  }

  // runs without the global lock: touches nothing shared but its own delay
  int switch_run(int i, bool, int) override {
    const int d = pending_delay_ms[i];
    if (d > 0) std::this_thread::sleep_for(std::chrono::milliseconds(d));
    return NOS_SMI_OK;
  }

  int switch_finish(int i, bool compute, int mode, int rc) override {
    switching[i] = 0;
    if (rc != NOS_SMI_OK) return rc;
    if (!stale_mode) (compute ? gpus[i].compute : gpus[i].memory) = mode;
    if (lose_after_switch) gpus[i].lost = true;
    // the session re-enumerates after its own switch (it then also sees any
    // external change of the other GPUs); GPUs still switching keep their view
    for (int j = 0; j < (int)gpus.size(); ++j)
      if (!is_switching(j)) view[j] = gpus[j];
    return NOS_SMI_OK;
  }

  int set_compute(int i, int mode) override {
    int rc = switch_prepare(i, true, mode);
    return rc ? rc : switch_finish(i, true, mode, switch_run(i, true, mode));
  }

  int set_memory(int i, int mode) override {
    int rc = switch_prepare(i, false, mode);
    return rc ? rc : switch_finish(i, false, mode, switch_run(i, false, mode));
  }

  int activity(int i, int* gfx, int* umc, int* mm) override {
    if (int rc = check(i)) return rc;
    *gfx = gpus[i].gfx;
    *umc = gpus[i].umc;
    *mm = 0;
    return NOS_SMI_OK;
  }

  int processes(int i, nos_proc_info* out, int max, int* n) override {
    if (int rc = check(i)) return rc;
    int k = 0;
    for (auto& kv : gpus[i].procs) {
      if (k < max) out[k] = kv.second;
      ++k;
    }
    *n = k;
    return NOS_SMI_OK;
  }

  int link(int i, int j, int* type, long long* hops, long long* weight) override {
    if (!ok(i) || !ok(j)) return NOS_SMI_ERR_BAD_INDEX;
    if (i == j) {
      *type = 0;
      *hops = 0;
      *weight = 0;
    } else {  // one 8-GPU MI355X node: fully connected xGMI mesh
      *type = 2;
      *hops = 1;
      *weight = 15;
    }
    return NOS_SMI_OK;
  }

  int clock(int i, int* cur, int* mx) override {
    if (int rc = check(i)) return rc;
    *mx = 2400;
    *cur = gpus[i].gfx > 0 ? 2400 : 500;  // busy GPUs run at the top clock, idle ones deep-sleep
    return NOS_SMI_OK;
  }

  // logical devices: GPU-major enumeration (the driver's order), partition p of
  // GPU i gets HIP id / render node after every partition of GPUs 0..i-1
  int partition_count(int i) override {
    if (int rc = check(i)) return rc;
    return partitions_for_mode(view[i].compute);
  }

  int partition_info(int i, int p, nos_part_info* o) override {
    if (int rc = check(i)) return rc;
    const FakeGpu& g = view[i];
    const int n = partitions_for_mode(g.compute);
    if (p < 0 || p >= n) return NOS_SMI_ERR_BAD_INDEX;
    int base = 0;
    for (int j = 0; j < i; ++j)
      if (!view[j].lost) base += partitions_for_mode(view[j].compute);
    std::memset(o, 0, sizeof(*o));
    o->gpu_index = i;
    o->partition = p;
    o->hip_id = base + p;
    o->drm_render = 128 + base + p;
    o->kfd_node = 1 + base + p;
    o->num_cus = g.cus / n;
    o->num_xcds = g.xcds / n > 0 ? g.xcds / n : 1;
    o->memory_shared = (g.memory == 1 && n > 1) ? 1 : 0;
    o->vram_mb = g.vram_mb / n;
    std::snprintf(o->bdf, sizeof(o->bdf), "0000:%02x:00.%d", 0x05 + 0x10 * i, p);
    std::snprintf(o->uuid, sizeof(o->uuid), "GPU-fake-mi355x-%04d-p%d", i, p);
    return NOS_SMI_OK;
  }

  int inject(const char* fault) override {
    std::string f(fault ? fault : "");
    if (f == "fail_set_compute") fail_set_compute = true;
    else if (f == "fail_set_memory") fail_set_memory = true;
    else if (f == "stale_mode") stale_mode = true;
    else if (f == "lose_after_switch") lose_after_switch = true;
    else if (f.rfind("switch_delay_ms=", 0) == 0) switch_delay_ms = std::stoi(f.substr(16));
    else if (f.rfind("lose_gpu=", 0) == 0) {
      int i = std::stoi(f.substr(9));
      if (i >= 0 && i < (int)gpus.size()) gpus[i].lost = view[i].lost = true;
    } else if (f.rfind("external_switch=", 0) == 0) {
      // "external_switch=<gpu>:<mode>": another process changed the GPU's compute
      // (SPX..CPX) or memory (NPSn) mode; this session sees it after rescan()
      const std::string arg = f.substr(16);
      const size_t c = arg.find(':');
      if (c == std::string::npos) return NOS_SMI_ERR_INVALID;
      const int i = std::stoi(arg.substr(0, c));
      const std::string m = arg.substr(c + 1);
      if (i < 0 || i >= (int)gpus.size()) return NOS_SMI_ERR_BAD_INDEX;
      if (int cm = parse_compute(m.c_str())) gpus[i].compute = cm;
      else if (int mm = parse_memory(m.c_str())) gpus[i].memory = mm;
      else return NOS_SMI_ERR_INVALID;
    } else if (f == "clear") {
      fail_set_compute = fail_set_memory = stale_mode = lose_after_switch = false;
      switch_delay_ms = 0;
      for (auto& g : gpus) g.lost = false;
      for (auto& g : view) g.lost = false;
    } else {
      return NOS_SMI_ERR_INVALID;
    }
    return NOS_SMI_OK;
  }

  int add_process(int i, unsigned pid, long long vram, unsigned cus) override {
    if (i < 0 || i >= (int)gpus.size() || gpus[i].lost) return NOS_SMI_ERR_BAD_INDEX;
    nos_proc_info p{};
    p.pid = pid;
    p.vram_bytes = vram;
    p.cu_occupancy = cus;
    std::snprintf(p.name, sizeof(p.name), "tenant-%u", pid);
    gpus[i].procs[pid] = p;
    return NOS_SMI_OK;
  }

  int remove_process(int i, unsigned pid) override {
    if (i < 0 || i >= (int)gpus.size() || gpus[i].lost) return NOS_SMI_ERR_BAD_INDEX;
    gpus[i].procs.erase(pid);
    return NOS_SMI_OK;
  }

  int set_activity(int i, int gfx, int umc) override {
    if (i < 0 || i >= (int)gpus.size() || gpus[i].lost) return NOS_SMI_ERR_BAD_INDEX;
    gpus[i].gfx = gfx;
    gpus[i].umc = umc;
    return NOS_SMI_OK;
  }
};

// ------------------------------------------------------------- amd-smi ----
struct SmiApi {
  void* h = nullptr;
#define NOS_SMI_FN(name) decltype(&::name) name = nullptr
  NOS_SMI_FN(amdsmi_init);
  NOS_SMI_FN(amdsmi_shut_down);
  NOS_SMI_FN(amdsmi_get_socket_handles);
  NOS_SMI_FN(amdsmi_get_processor_handles);
  NOS_SMI_FN(amdsmi_get_gpu_asic_info);
  NOS_SMI_FN(amdsmi_get_gpu_vram_info);
  NOS_SMI_FN(amdsmi_get_gpu_device_bdf);
  NOS_SMI_FN(amdsmi_get_gpu_device_uuid);
  NOS_SMI_FN(amdsmi_get_gpu_enumeration_info);
  NOS_SMI_FN(amdsmi_get_gpu_xcd_counter);
  NOS_SMI_FN(amdsmi_get_gpu_compute_partition);
  NOS_SMI_FN(amdsmi_set_gpu_compute_partition);
  NOS_SMI_FN(amdsmi_get_gpu_memory_partition);
  NOS_SMI_FN(amdsmi_set_gpu_memory_partition);
  NOS_SMI_FN(amdsmi_get_gpu_activity);
  NOS_SMI_FN(amdsmi_get_gpu_process_list);
  NOS_SMI_FN(amdsmi_topo_get_link_type);
  NOS_SMI_FN(amdsmi_topo_get_link_weight);
  NOS_SMI_FN(amdsmi_get_gpu_kfd_info);
  NOS_SMI_FN(amdsmi_get_clock_info);
#undef NOS_SMI_FN

  bool load() {
    const char* names[] = {"libamd_smi.so", "libamd_smi.so.26", "/opt/rocm/lib/libamd_smi.so"};
    for (const char* n : names) {
      h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) return false;
#define NOS_SMI_LOAD(name) name = reinterpret_cast<decltype(name)>(dlsym(h, #name))
    NOS_SMI_LOAD(amdsmi_init);
    NOS_SMI_LOAD(amdsmi_shut_down);
    NOS_SMI_LOAD(amdsmi_get_socket_handles);
    NOS_SMI_LOAD(amdsmi_get_processor_handles);
    NOS_SMI_LOAD(amdsmi_get_gpu_asic_info);
    NOS_SMI_LOAD(amdsmi_get_gpu_vram_info);
    NOS_SMI_LOAD(amdsmi_get_gpu_device_bdf);
    NOS_SMI_LOAD(amdsmi_get_gpu_device_uuid);
    NOS_SMI_LOAD(amdsmi_get_gpu_enumeration_info);
    NOS_SMI_LOAD(amdsmi_get_gpu_xcd_counter);
    NOS_SMI_LOAD(amdsmi_get_gpu_compute_partition);
    NOS_SMI_LOAD(amdsmi_set_gpu_compute_partition);
    NOS_SMI_LOAD(amdsmi_get_gpu_memory_partition);
    NOS_SMI_LOAD(amdsmi_set_gpu_memory_partition);
    NOS_SMI_LOAD(amdsmi_get_gpu_activity);
    NOS_SMI_LOAD(amdsmi_get_gpu_process_list);
    NOS_SMI_LOAD(amdsmi_topo_get_link_type);
    NOS_SMI_LOAD(amdsmi_topo_get_link_weight);
    NOS_SMI_LOAD(amdsmi_get_gpu_kfd_info);
    NOS_SMI_LOAD(amdsmi_get_clock_info);
#undef NOS_SMI_LOAD
    return amdsmi_init && amdsmi_get_socket_handles && amdsmi_get_processor_handles;
  }
};

struct AmdSmiBackend : Backend {
  SmiApi api;
  // physical GPU -> its processor handles (one per logical partition, ordered
  // by KFD partition id; SPX: exactly one)
  std::vector<std::vector<amdsmi_processor_handle>> gpus;
  std::vector<amdsmi_processor_handle> pending;  // per GPU: handle an in-flight switch was issued on
  bool allow_set = false;
  bool need_rescan = false;  // a switch finished while another was in flight

  int open(bool allow_set_) {
    allow_set = allow_set_;
    if (!api.load()) return NOS_SMI_ERR_BACKEND;
    if (api.amdsmi_init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return NOS_SMI_ERR_BACKEND;
    return enumerate();
  }

  uint32_t partition_id(amdsmi_processor_handle h) {
    amdsmi_kfd_info_t kfd{};
    if (api.amdsmi_get_gpu_kfd_info && api.amdsmi_get_gpu_kfd_info(h, &kfd) == AMDSMI_STATUS_SUCCESS &&
        kfd.current_partition_id != 0xFFFFFFFFu)
      return kfd.current_partition_id;
    amdsmi_bdf_t bdf{};
    if (api.amdsmi_get_gpu_device_bdf && api.amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS)
      return (uint32_t)bdf.function_number;
    return 0;
  }

  // one amd-smi socket = one physical device (its PCI bus/device); a socket
  // lists the processor handles of every partition the current mode exposes
  int enumerate() {
    gpus.clear();
    need_rescan = false;
    uint32_t ns = 0;
    if (api.amdsmi_get_socket_handles(&ns, nullptr) != AMDSMI_STATUS_SUCCESS) return NOS_SMI_ERR_BACKEND;
    std::vector<amdsmi_socket_handle> sockets(ns);
    if (ns && api.amdsmi_get_socket_handles(&ns, sockets.data()) != AMDSMI_STATUS_SUCCESS) return NOS_SMI_ERR_BACKEND;
    for (uint32_t s = 0; s < ns; ++s) {
      uint32_t np = 0;
      if (api.amdsmi_get_processor_handles(sockets[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
      std::vector<amdsmi_processor_handle> ph(np);
      if (api.amdsmi_get_processor_handles(sockets[s], &np, ph.data()) != AMDSMI_STATUS_SUCCESS) continue;
      ph.resize(np);
      std::vector<std::pair<uint32_t, amdsmi_processor_handle>> keyed;
      for (auto h : ph) keyed.emplace_back(partition_id(h), h);
      std::stable_sort(keyed.begin(), keyed.end(),
                       [](const auto& x, const auto& y) { return x.first < y.first; });
      std::vector<amdsmi_processor_handle> parts;
      for (auto& kv : keyed) parts.push_back(kv.second);
      gpus.push_back(parts);
    }
    switching.assign(gpus.size(), 0);
    pending.assign(gpus.size(), nullptr);
    return NOS_SMI_OK;
  }

  bool any_switching() const {
    for (char c : switching)
      if (c) return true;
    return false;
  }

  // shut the session down and enumerate again: invalidates every handle, so
  // never while a switch (holding a captured handle) is in flight
  int reinit() {
    if (any_switching()) return NOS_SMI_ERR_SWITCHING;
    if (api.amdsmi_shut_down) api.amdsmi_shut_down();
    if (api.amdsmi_init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return NOS_SMI_ERR_BACKEND;
    return enumerate();
  }

  int rescan() override { return reinit(); }

  int check(int i) const {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    return is_switching(i) ? NOS_SMI_ERR_SWITCHING : NOS_SMI_OK;
  }

  ~AmdSmiBackend() override {
    if (api.amdsmi_shut_down) api.amdsmi_shut_down();
    if (api.h) dlclose(api.h);
  }

  bool ok(int i) const { return i >= 0 && i < (int)gpus.size() && !gpus[i].empty(); }

  int count() override { return (int)gpus.size(); }

  long long vram_mb(amdsmi_processor_handle h) {
    amdsmi_vram_info_t vram{};
    if (api.amdsmi_get_gpu_vram_info && api.amdsmi_get_gpu_vram_info(h, &vram) == AMDSMI_STATUS_SUCCESS)
      return (long long)vram.vram_size;
    return 0;
  }

  int cus(amdsmi_processor_handle h) {
    amdsmi_asic_info_t asic{};
    if (api.amdsmi_get_gpu_asic_info && api.amdsmi_get_gpu_asic_info(h, &asic) == AMDSMI_STATUS_SUCCESS)
      return asic.num_of_compute_units == 0xFFFFFFFFu ? 0 : (int)asic.num_of_compute_units;
    return 0;
  }

  int xcds(amdsmi_processor_handle h) {
    uint16_t x = 0;
    if (api.amdsmi_get_gpu_xcd_counter && api.amdsmi_get_gpu_xcd_counter(h, &x) == AMDSMI_STATUS_SUCCESS) return x;
    return 0;
  }

  int memory_mode(amdsmi_processor_handle h) {
    char buf[64] = {0};
    if (api.amdsmi_get_gpu_memory_partition &&
        api.amdsmi_get_gpu_memory_partition(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS)
      return parse_memory(buf);
    return 0;
  }

  // total memory of the physical GPU: in NPS1 every partition sees the whole
  // pool, in NPSn each sees its NUMA range
  long long total_vram_mb(int i) {
    const auto& parts = gpus[i];
    long long mx = 0, sum = 0;
    for (auto h : parts) {
      const long long v = vram_mb(h);
      mx = v > mx ? v : mx;
      sum += v;
    }
    return (parts.size() > 1 && memory_mode(parts[0]) != 1) ? sum : mx;
  }

  int info(int i, nos_gpu_info* o) override {
    if (int rc = check(i)) return rc;
    std::memset(o, 0, sizeof(*o));
    const auto& parts = gpus[i];
    auto h = parts[0];
    o->index = i;
    o->hip_id = -1;
    o->drm_render = -1;
    amdsmi_asic_info_t asic{};
    if (api.amdsmi_get_gpu_asic_info && api.amdsmi_get_gpu_asic_info(h, &asic) == AMDSMI_STATUS_SUCCESS)
      std::snprintf(o->market_name, sizeof(o->market_name), "%s", asic.market_name);
    for (auto ph : parts) {
      o->num_cus += cus(ph);
      o->num_xcds += xcds(ph);
    }
    o->vram_mb = total_vram_mb(i);
    amdsmi_bdf_t bdf{};
    if (api.amdsmi_get_gpu_device_bdf && api.amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS)
      std::snprintf(o->bdf, sizeof(o->bdf), "%04llx:%02x:%02x.%x",
                    (unsigned long long)bdf.domain_number, (unsigned)bdf.bus_number,
                    (unsigned)bdf.device_number, (unsigned)bdf.function_number);
    unsigned ulen = sizeof(o->uuid);
    if (api.amdsmi_get_gpu_device_uuid) api.amdsmi_get_gpu_device_uuid(h, &ulen, o->uuid);
    amdsmi_enumeration_info_t en{};
    if (api.amdsmi_get_gpu_enumeration_info &&
        api.amdsmi_get_gpu_enumeration_info(h, &en) == AMDSMI_STATUS_SUCCESS) {
      o->hip_id = (int)en.hip_id;
      o->drm_render = (int)en.drm_render;
    }
    char buf[64] = {0};
    if (api.amdsmi_get_gpu_compute_partition &&
        api.amdsmi_get_gpu_compute_partition(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS)
      o->compute_mode = parse_compute(buf);
    o->memory_mode = memory_mode(h);
    o->num_partitions = (int)parts.size() > 1 ? (int)parts.size() : partitions_for_mode(o->compute_mode);
    return NOS_SMI_OK;
  }

  int partition_count(int i) override {
    if (int rc = check(i)) return rc;
    return (int)gpus[i].size();
  }

  int clock(int i, int* cur, int* mx) override {
    if (int rc = check(i)) return rc;
    if (!api.amdsmi_get_clock_info) return NOS_SMI_ERR_UNSUPPORTED;
    amdsmi_clk_info_t c{};
    if (api.amdsmi_get_clock_info(gpus[i][0], AMDSMI_CLK_TYPE_GFX, &c) != AMDSMI_STATUS_SUCCESS)
      return NOS_SMI_ERR_BACKEND;
    *cur = (int)c.clk;
    *mx = (int)c.max_clk;
    return NOS_SMI_OK;
  }

  int partition_info(int i, int p, nos_part_info* o) override {
    if (int rc = check(i)) return rc;
    const auto& parts = gpus[i];
    if (p < 0 || p >= (int)parts.size()) return NOS_SMI_ERR_BAD_INDEX;
    auto h = parts[p];
    std::memset(o, 0, sizeof(*o));
    o->gpu_index = i;
    o->partition = p;
    o->hip_id = -1;
    o->drm_render = -1;
    o->kfd_node = -1;
    amdsmi_enumeration_info_t en{};
    if (api.amdsmi_get_gpu_enumeration_info &&
        api.amdsmi_get_gpu_enumeration_info(h, &en) == AMDSMI_STATUS_SUCCESS) {
      o->hip_id = (int)en.hip_id;
      o->drm_render = (int)en.drm_render;
    }
    amdsmi_kfd_info_t kfd{};
    if (api.amdsmi_get_gpu_kfd_info && api.amdsmi_get_gpu_kfd_info(h, &kfd) == AMDSMI_STATUS_SUCCESS &&
        kfd.node_id != 0xFFFFFFFFu)
      o->kfd_node = (int)kfd.node_id;
    o->num_cus = cus(h);
    o->num_xcds = xcds(h);
    const int n = (int)parts.size();
    o->memory_shared = (n > 1 && memory_mode(h) == 1) ? 1 : 0;
    o->vram_mb = o->memory_shared ? total_vram_mb(i) / n : vram_mb(h);
    amdsmi_bdf_t bdf{};
    if (api.amdsmi_get_gpu_device_bdf && api.amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS)
      std::snprintf(o->bdf, sizeof(o->bdf), "%04llx:%02x:%02x.%x",
                    (unsigned long long)bdf.domain_number, (unsigned)bdf.bus_number,
                    (unsigned)bdf.device_number, (unsigned)bdf.function_number);
    unsigned ulen = sizeof(o->uuid);
    if (api.amdsmi_get_gpu_device_uuid) api.amdsmi_get_gpu_device_uuid(h, &ulen, o->uuid);
    return NOS_SMI_OK;
  }

  // a mode switch is GPU-wide: issued on the first partition's handle; the
  // handle set changes with the mode, so the session re-enumerates afterwards
  int switch_prepare(int i, bool compute, int mode) override {
    if (int rc = check(i)) return rc;
    if (compute ? !api.amdsmi_set_gpu_compute_partition : !api.amdsmi_set_gpu_memory_partition)
      return NOS_SMI_ERR_UNSUPPORTED;
    if (!allow_set) return NOS_SMI_ERR_UNSUPPORTED;
    int n = 0;
    nos_proc_info tmp[1];
    if (processes(i, tmp, 1, &n) == NOS_SMI_OK && n > 0) return NOS_SMI_ERR_BUSY;
    pending[i] = gpus[i][0];
    switching[i] = 1;
    return NOS_SMI_OK;
  }

  int switch_run(int i, bool compute, int mode) override {
    auto h = pending[i];
    auto st = compute ? api.amdsmi_set_gpu_compute_partition(h, (amdsmi_compute_partition_type_t)mode)
                      : api.amdsmi_set_gpu_memory_partition(h, (amdsmi_memory_partition_type_t)mode);
    return st == AMDSMI_STATUS_SUCCESS ? NOS_SMI_OK : NOS_SMI_ERR_BACKEND;
  }

  int switch_finish(int i, bool, int, int rc) override {
    switching[i] = 0;
    pending[i] = nullptr;
    if (any_switching()) {  // handles are still in use by another switch: re-enumerate when it ends
      need_rescan = true;
      return rc;
    }
    const int rs = reinit();
    return rc != NOS_SMI_OK ? rc : rs;
  }

  int set_compute(int i, int mode) override {
    int rc = switch_prepare(i, true, mode);
    return rc ? rc : switch_finish(i, true, mode, switch_run(i, true, mode));
  }

  int set_memory(int i, int mode) override {
    int rc = switch_prepare(i, false, mode);
    return rc ? rc : switch_finish(i, false, mode, switch_run(i, false, mode));
  }

  int activity(int i, int* gfx, int* umc, int* mm) override {
    if (int rc = check(i)) return rc;
    if (!api.amdsmi_get_gpu_activity) return NOS_SMI_ERR_UNSUPPORTED;
    amdsmi_engine_usage_t u{};
    if (api.amdsmi_get_gpu_activity(gpus[i][0], &u) != AMDSMI_STATUS_SUCCESS) return NOS_SMI_ERR_BACKEND;
    *gfx = (int)u.gfx_activity;
    *umc = (int)u.umc_activity;
    *mm = (int)u.mm_activity;
    return NOS_SMI_OK;
  }

  // processes of every partition of the GPU (a repartition drains them all)
  int processes(int i, nos_proc_info* out, int max, int* n) override {
    if (int rc = check(i)) return rc;
    if (!api.amdsmi_get_gpu_process_list) return NOS_SMI_ERR_UNSUPPORTED;
    std::map<unsigned, nos_proc_info> seen;
    for (auto h : gpus[i]) {
      std::vector<amdsmi_proc_info_t> buf(64);
      uint32_t cnt = (uint32_t)buf.size();
      auto st = api.amdsmi_get_gpu_process_list(h, &cnt, buf.data());
      if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) return NOS_SMI_ERR_BACKEND;
      for (uint32_t p = 0; p < cnt && p < buf.size(); ++p) {
        nos_proc_info& q = seen[buf[p].pid];
        q.pid = buf[p].pid;
        q.cu_occupancy += buf[p].cu_occupancy;
        q.vram_bytes += (long long)buf[p].memory_usage.vram_mem;
        std::snprintf(q.name, sizeof(q.name), "%s", buf[p].name);
      }
    }
    int k = 0;
    for (auto& kv : seen) {
      if (k < max) out[k] = kv.second;
      ++k;
    }
    *n = k;
    return NOS_SMI_OK;
  }

  int link(int i, int j, int* type, long long* hops, long long* weight) override {
    if (!ok(i) || !ok(j)) return NOS_SMI_ERR_BAD_INDEX;
    if (i == j) {
      *type = 0;
      *hops = 0;
      *weight = 0;
      return NOS_SMI_OK;
    }
    if (is_switching(i) || is_switching(j)) return NOS_SMI_ERR_SWITCHING;
    if (!api.amdsmi_topo_get_link_type) return NOS_SMI_ERR_UNSUPPORTED;
    uint64_t h = 0, w = 0;
    amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
    if (api.amdsmi_topo_get_link_type(gpus[i][0], gpus[j][0], &h, &t) != AMDSMI_STATUS_SUCCESS)
      return NOS_SMI_ERR_BACKEND;
    if (api.amdsmi_topo_get_link_weight) api.amdsmi_topo_get_link_weight(gpus[i][0], gpus[j][0], &w);
    *type = (int)t;
    *hops = (long long)h;
    *weight = (long long)w;
    return NOS_SMI_OK;
  }
};

std::mutex g_mu;
// Deliberately a heap object that is never destroyed by static destructors:
// amd-smi tears its own singletons down at exit, and shutting it down again from
// our destructor afterwards segfaults (seen on MI355X, ROCm 7.2).  Explicit
// nos_smi_close() releases the session (an in-flight mode switch keeps its
// backend alive through its own reference until it returns).
std::shared_ptr<Backend>& g_backend = *new std::shared_ptr<Backend>();

void set_backend(Backend* b) { g_backend.reset(b); }

int do_switch(int i, bool compute, int mode) {
  std::shared_ptr<Backend> b;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_backend) return NOS_SMI_ERR_NOT_OPEN;
    b = g_backend;
    if (int rc = b->switch_prepare(i, compute, mode)) return rc;
  }
  const int rc = b->switch_run(i, compute, mode);  // the slow part: no global lock
  std::lock_guard<std::mutex> lk(g_mu);
  return b->switch_finish(i, compute, mode, rc);
}

}  // namespace

// backend: "fake" or "amdsmi". spec: fake node description (see FakeBackend).
// allow_set: the amd-smi setters are refused unless explicitly enabled.
NOS_API int nos_smi_open(const char* backend, const char* spec, int allow_set) {
  std::lock_guard<std::mutex> lk(g_mu);
  std::string b(backend ? backend : "amdsmi");
  if (b == "fake") {
    set_backend(new FakeBackend(spec ? spec : ""));
    return NOS_SMI_OK;
  }
  auto* real = new AmdSmiBackend();
  int rc = real->open(allow_set != 0);
  if (rc != NOS_SMI_OK) {
    delete real;
    set_backend(nullptr);
    return rc;
  }
  set_backend(real);
  return NOS_SMI_OK;
}

NOS_API int nos_smi_close() {
  std::lock_guard<std::mutex> lk(g_mu);
  set_backend(nullptr);
  return NOS_SMI_OK;
}

#define NOS_SMI_GUARD()                          \
  std::lock_guard<std::mutex> lk(g_mu);          \
  if (!g_backend) return NOS_SMI_ERR_NOT_OPEN

NOS_API int nos_smi_count() {
  NOS_SMI_GUARD();
  return g_backend->count();
}
NOS_API int nos_smi_gpu_info(int i, nos_gpu_info* out) {
  NOS_SMI_GUARD();
  return g_backend->info(i, out);
}
NOS_API int nos_smi_set_compute_partition(int i, int mode) { return do_switch(i, true, mode); }
NOS_API int nos_smi_set_memory_partition(int i, int mode) { return do_switch(i, false, mode); }
// re-enumerate (modes switched by another process become visible);
// NOS_SMI_ERR_SWITCHING while one of this session's switches is in flight
NOS_API int nos_smi_rescan() {
  NOS_SMI_GUARD();
  return g_backend->rescan();
}
NOS_API int nos_smi_activity(int i, int* gfx, int* umc, int* mm) {
  NOS_SMI_GUARD();
  return g_backend->activity(i, gfx, umc, mm);
}
NOS_API int nos_smi_processes(int i, nos_proc_info* out, int max, int* n) {
  NOS_SMI_GUARD();
  return g_backend->processes(i, out, max, n);
}
NOS_API int nos_smi_link(int i, int j, int* type, long long* hops, long long* weight) {
  NOS_SMI_GUARD();
  return g_backend->link(i, j, type, hops, weight);
}
NOS_API int nos_smi_clock(int i, int* cur_mhz, int* max_mhz) {
  NOS_SMI_GUARD();
  return g_backend->clock(i, cur_mhz, max_mhz);
}
NOS_API int nos_smi_partition_count(int i) {
  NOS_SMI_GUARD();
  return g_backend->partition_count(i);
}
NOS_API int nos_smi_partition_info(int i, int p, nos_part_info* out) {
  NOS_SMI_GUARD();
  return g_backend->partition_info(i, p, out);
}
NOS_API int nos_smi_fake_inject(const char* fault) {
  NOS_SMI_GUARD();
  return g_backend->inject(fault);
}
NOS_API int nos_smi_fake_add_process(int i, unsigned pid, long long vram, unsigned cus) {
  NOS_SMI_GUARD();
  return g_backend->add_process(i, pid, vram, cus);
}
NOS_API int nos_smi_fake_remove_process(int i, unsigned pid) {
  NOS_SMI_GUARD();
  return g_backend->remove_process(i, pid);
}
NOS_API int nos_smi_fake_set_activity(int i, int gfx, int umc) {
  NOS_SMI_GUARD();
  return g_backend->set_activity(i, gfx, umc);
}
NOS_API int nos_smi_struct_sizes(int* gpu_info, int* proc_info) {
  *gpu_info = (int)sizeof(nos_gpu_info);
  *proc_info = (int)sizeof(nos_proc_info);
  return NOS_SMI_OK;
}
NOS_API int nos_smi_part_struct_size() { return (int)sizeof(nos_part_info); }
