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
// All entry points are serialised by one mutex (the reference's NVML client
// does Init/Shutdown per call, client.go:46-57; we keep one session open).
#include <dlfcn.h>

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
  std::vector<FakeGpu> gpus;
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
  }

  bool ok(int i) const { return i >= 0 && i < (int)gpus.size() && !gpus[i].lost; }

  int count() override { return (int)gpus.size(); }

  int info(int i, nos_gpu_info* o) override {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    const FakeGpu& g = gpus[i];
    std::memset(o, 0, sizeof(*o));
    o->index = i;
    o->num_cus = g.cus;
    o->num_xcds = g.xcds;
    o->compute_mode = g.compute;
    o->memory_mode = g.memory;
    o->num_partitions = partitions_for_mode(g.compute);
    o->hip_id = i;
    o->drm_render = 128 + i;
    o->vram_mb = g.vram_mb;
    std::snprintf(o->bdf, sizeof(o->bdf), "0000:%02x:00.0", 0x05 + 0x10 * i);
    std::snprintf(o->uuid, sizeof(o->uuid), "GPU-fake-mi355x-%04d", i);
    std::snprintf(o->market_name, sizeof(o->market_name), "%s", model.c_str());
    return NOS_SMI_OK;
  }

  int set_mode_common(int i, int* field, int mode, bool fail) {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    if (fail) return NOS_SMI_ERR_INJECTED;
    if (!gpus[i].procs.empty()) return NOS_SMI_ERR_BUSY;
    if (switch_delay_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(switch_delay_ms));
    if (!stale_mode) *field = mode;
    if (lose_after_switch) gpus[i].lost = true;
    return NOS_SMI_OK;
  }

  int set_compute(int i, int mode) override {
    if (mode < 1 || mode > 5) return NOS_SMI_ERR_INVALID;
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    return set_mode_common(i, &gpus[i].compute, mode, fail_set_compute);
  }

  int set_memory(int i, int mode) override {
    if (mode != 1 && mode != 2 && mode != 4 && mode != 8) return NOS_SMI_ERR_INVALID;
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    return set_mode_common(i, &gpus[i].memory, mode, fail_set_memory);
  }

  int activity(int i, int* gfx, int* umc, int* mm) override {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    *gfx = gpus[i].gfx;
    *umc = gpus[i].umc;
    *mm = 0;
    return NOS_SMI_OK;
  }

  int processes(int i, nos_proc_info* out, int max, int* n) override {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
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

  int inject(const char* fault) override {
    std::string f(fault ? fault : "");
    if (f == "fail_set_compute") fail_set_compute = true;
    else if (f == "fail_set_memory") fail_set_memory = true;
    else if (f == "stale_mode") stale_mode = true;
    else if (f == "lose_after_switch") lose_after_switch = true;
    else if (f.rfind("switch_delay_ms=", 0) == 0) switch_delay_ms = std::stoi(f.substr(16));
    else if (f.rfind("lose_gpu=", 0) == 0) {
      int i = std::stoi(f.substr(9));
      if (i >= 0 && i < (int)gpus.size()) gpus[i].lost = true;
    } else if (f == "clear") {
      fail_set_compute = fail_set_memory = stale_mode = lose_after_switch = false;
      switch_delay_ms = 0;
      for (auto& g : gpus) g.lost = false;
    } else {
      return NOS_SMI_ERR_INVALID;
    }
    return NOS_SMI_OK;
  }

  int add_process(int i, unsigned pid, long long vram, unsigned cus) override {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    nos_proc_info p{};
    p.pid = pid;
    p.vram_bytes = vram;
    p.cu_occupancy = cus;
    std::snprintf(p.name, sizeof(p.name), "tenant-%u", pid);
    gpus[i].procs[pid] = p;
    return NOS_SMI_OK;
  }

  int remove_process(int i, unsigned pid) override {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    gpus[i].procs.erase(pid);
    return NOS_SMI_OK;
  }

  int set_activity(int i, int gfx, int umc) override {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
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
#undef NOS_SMI_LOAD
    return amdsmi_init && amdsmi_get_socket_handles && amdsmi_get_processor_handles;
  }
};

struct AmdSmiBackend : Backend {
  SmiApi api;
  std::vector<amdsmi_processor_handle> handles;
  bool allow_set = false;

  int open(bool allow_set_) {
    allow_set = allow_set_;
    if (!api.load()) return NOS_SMI_ERR_BACKEND;
    if (api.amdsmi_init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return NOS_SMI_ERR_BACKEND;
    uint32_t ns = 0;
    if (api.amdsmi_get_socket_handles(&ns, nullptr) != AMDSMI_STATUS_SUCCESS) return NOS_SMI_ERR_BACKEND;
    std::vector<amdsmi_socket_handle> sockets(ns);
    if (ns && api.amdsmi_get_socket_handles(&ns, sockets.data()) != AMDSMI_STATUS_SUCCESS)
      return NOS_SMI_ERR_BACKEND;
    for (uint32_t s = 0; s < ns; ++s) {
      uint32_t np = 0;
      if (api.amdsmi_get_processor_handles(sockets[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
      std::vector<amdsmi_processor_handle> ph(np);
      if (np && api.amdsmi_get_processor_handles(sockets[s], &np, ph.data()) == AMDSMI_STATUS_SUCCESS)
        handles.insert(handles.end(), ph.begin(), ph.begin() + np);
    }
    return NOS_SMI_OK;
  }

  ~AmdSmiBackend() override {
    if (api.amdsmi_shut_down) api.amdsmi_shut_down();
    if (api.h) dlclose(api.h);
  }

  bool ok(int i) const { return i >= 0 && i < (int)handles.size(); }

  int count() override { return (int)handles.size(); }

  int info(int i, nos_gpu_info* o) override {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    std::memset(o, 0, sizeof(*o));
    auto h = handles[i];
    o->index = i;
    o->hip_id = -1;
    o->drm_render = -1;
    amdsmi_asic_info_t asic{};
    if (api.amdsmi_get_gpu_asic_info && api.amdsmi_get_gpu_asic_info(h, &asic) == AMDSMI_STATUS_SUCCESS) {
      std::snprintf(o->market_name, sizeof(o->market_name), "%s", asic.market_name);
      o->num_cus = asic.num_of_compute_units == 0xFFFFFFFFu ? 0 : (int)asic.num_of_compute_units;
    }
    amdsmi_vram_info_t vram{};
    if (api.amdsmi_get_gpu_vram_info && api.amdsmi_get_gpu_vram_info(h, &vram) == AMDSMI_STATUS_SUCCESS)
      o->vram_mb = (long long)vram.vram_size;
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
    uint16_t xcd = 0;
    if (api.amdsmi_get_gpu_xcd_counter && api.amdsmi_get_gpu_xcd_counter(h, &xcd) == AMDSMI_STATUS_SUCCESS)
      o->num_xcds = xcd;
    char buf[64] = {0};
    if (api.amdsmi_get_gpu_compute_partition &&
        api.amdsmi_get_gpu_compute_partition(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS)
      o->compute_mode = parse_compute(buf);
    std::memset(buf, 0, sizeof(buf));
    if (api.amdsmi_get_gpu_memory_partition &&
        api.amdsmi_get_gpu_memory_partition(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS)
      o->memory_mode = parse_memory(buf);
    o->num_partitions = partitions_for_mode(o->compute_mode);
    return NOS_SMI_OK;
  }

  int set_compute(int i, int mode) override {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    if (!allow_set || !api.amdsmi_set_gpu_compute_partition) return NOS_SMI_ERR_UNSUPPORTED;
    int n = 0;
    nos_proc_info tmp[1];
    if (processes(i, tmp, 1, &n) == NOS_SMI_OK && n > 0) return NOS_SMI_ERR_BUSY;
    auto st = api.amdsmi_set_gpu_compute_partition(handles[i], (amdsmi_compute_partition_type_t)mode);
    return st == AMDSMI_STATUS_SUCCESS ? NOS_SMI_OK : NOS_SMI_ERR_BACKEND;
  }

  int set_memory(int i, int mode) override {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    if (!allow_set || !api.amdsmi_set_gpu_memory_partition) return NOS_SMI_ERR_UNSUPPORTED;
    int n = 0;
    nos_proc_info tmp[1];
    if (processes(i, tmp, 1, &n) == NOS_SMI_OK && n > 0) return NOS_SMI_ERR_BUSY;
    auto st = api.amdsmi_set_gpu_memory_partition(handles[i], (amdsmi_memory_partition_type_t)mode);
    return st == AMDSMI_STATUS_SUCCESS ? NOS_SMI_OK : NOS_SMI_ERR_BACKEND;
  }

  int activity(int i, int* gfx, int* umc, int* mm) override {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    if (!api.amdsmi_get_gpu_activity) return NOS_SMI_ERR_UNSUPPORTED;
    amdsmi_engine_usage_t u{};
    if (api.amdsmi_get_gpu_activity(handles[i], &u) != AMDSMI_STATUS_SUCCESS) return NOS_SMI_ERR_BACKEND;
    *gfx = (int)u.gfx_activity;
    *umc = (int)u.umc_activity;
    *mm = (int)u.mm_activity;
    return NOS_SMI_OK;
  }

  int processes(int i, nos_proc_info* out, int max, int* n) override {
    if (!ok(i)) return NOS_SMI_ERR_BAD_INDEX;
    if (!api.amdsmi_get_gpu_process_list) return NOS_SMI_ERR_UNSUPPORTED;
    uint32_t cnt = 0;
    std::vector<amdsmi_proc_info_t> buf(64);
    cnt = (uint32_t)buf.size();
    auto st = api.amdsmi_get_gpu_process_list(handles[i], &cnt, buf.data());
    if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) return NOS_SMI_ERR_BACKEND;
    int k = 0;
    for (uint32_t p = 0; p < cnt && p < buf.size(); ++p) {
      if (k < max) {
        out[k].pid = buf[p].pid;
        out[k].cu_occupancy = buf[p].cu_occupancy;
        out[k].vram_bytes = (long long)buf[p].memory_usage.vram_mem;
        std::snprintf(out[k].name, sizeof(out[k].name), "%s", buf[p].name);
      }
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
    if (!api.amdsmi_topo_get_link_type) return NOS_SMI_ERR_UNSUPPORTED;
    uint64_t h = 0, w = 0;
    amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
    if (api.amdsmi_topo_get_link_type(handles[i], handles[j], &h, &t) != AMDSMI_STATUS_SUCCESS)
      return NOS_SMI_ERR_BACKEND;
    if (api.amdsmi_topo_get_link_weight) api.amdsmi_topo_get_link_weight(handles[i], handles[j], &w);
    *type = (int)t;
    *hops = (long long)h;
    *weight = (long long)w;
    return NOS_SMI_OK;
  }
};

std::mutex g_mu;
// Deliberately a raw pointer that is never destroyed by static destructors:
// amd-smi tears its own singletons down at exit, and shutting it down again from
// our destructor afterwards segfaults (seen on MI355X, ROCm 7.2).  Explicit
// nos_smi_close() releases the session.
Backend* g_backend = nullptr;

void set_backend(Backend* b) {
  delete g_backend;
  g_backend = b;
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
NOS_API int nos_smi_set_compute_partition(int i, int mode) {
  NOS_SMI_GUARD();
  return g_backend->set_compute(i, mode);
}
NOS_API int nos_smi_set_memory_partition(int i, int mode) {
  NOS_SMI_GUARD();
  return g_backend->set_memory(i, mode);
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
