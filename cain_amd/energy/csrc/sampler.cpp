// Native energy / utilisation sampler for the MI355X energy harness.
//
// Replaces the reference's measurement substrate:
//   * `sudo powermetrics -i 100 --samplers gpu_power` GPU residency
//     (reference experiment/RunnerConfig.py:140-143, parsed :207-226),
//   * codecarbon's OfflineEmissionsTracker whole-machine energy estimate
//     (reference experiment-runner/Plugins/Profilers/CodecarbonWrapper.py:43-68),
//   * the psutil cpu%/mem% loop (reference experiment/RunnerConfig.py:156-173).
//
// Design: one sampler thread pinned to a core polls the amd-smi GPU energy
// accumulator every `fast_period_us` (default 1 ms) and records a
// (host time, cumulative joules) point only when the accumulator moves (the
// firmware updates it every ~10-20 ms on MI355X).  Window energy is then an
// interpolation on that piecewise-linear trace, so windows far shorter than
// the counter cadence still integrate correctly (the reference's remote-arm
// energies sit on a ~6.8 J lattice).  Every `period_us` (default
// 100 ms, powermetrics' cadence) it also takes a slow sample: board power,
// gfx/umc activity, VRAM %, host CPU % (/proc/stat deltas), host memory %
// (/proc/meminfo, psutil's formula) and the host CPU energy counter when one
// is readable (HostEnergy below: amd-smi CPU sockets via HSMP, else RAPL
// powercap package zones, else hwmon `amd_energy` socket sensors), accumulated
// per counter with modular wrap handling.  libamd_smi is dlopen'ed so the
// library loads (and the CPU-side metrics work) on hosts without a GPU.
//
// Exposed as a plain C ABI consumed through ctypes (cain_amd/energy/native.py).

#include <amd_smi/amdsmi.h>
#include <dlfcn.h>
#include <pthread.h>
#include <sys/syscall.h>
#include <sched.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <dirent.h>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

using fn_init_t = amdsmi_status_t (*)(uint64_t);
using fn_shutdown_t = amdsmi_status_t (*)();
using fn_sockets_t = amdsmi_status_t (*)(uint32_t*, amdsmi_socket_handle*);
using fn_procs_t = amdsmi_status_t (*)(amdsmi_socket_handle, uint32_t*, amdsmi_processor_handle*);
using fn_energy_t = amdsmi_status_t (*)(amdsmi_processor_handle, uint64_t*, float*, uint64_t*);
using fn_power_t = amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_power_info_t*);
using fn_activity_t = amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_engine_usage_t*);
using fn_vram_t = amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_vram_usage_t*);
using fn_bdf_t = amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_bdf_t*);
using fn_type_t = amdsmi_status_t (*)(amdsmi_processor_handle, processor_type_t*);
using fn_cpu_handles_t = amdsmi_status_t (*)(uint32_t*, amdsmi_processor_handle*);
using fn_cpu_energy_t = amdsmi_status_t (*)(amdsmi_processor_handle, uint64_t*);

struct Smi {
  void* lib = nullptr;
  fn_init_t init = nullptr;
  fn_shutdown_t shutdown = nullptr;
  fn_sockets_t sockets = nullptr;
  fn_procs_t procs = nullptr;
  fn_energy_t energy = nullptr;
  fn_power_t power = nullptr;
  fn_activity_t activity = nullptr;
  fn_vram_t vram = nullptr;
  fn_bdf_t bdf = nullptr;
  fn_type_t ptype = nullptr;
  fn_cpu_handles_t cpu_handles = nullptr;
  fn_cpu_energy_t cpu_energy = nullptr;
  std::vector<amdsmi_processor_handle> gpus;
  std::vector<amdsmi_processor_handle> cpus;  // CPU sockets (only when the HSMP driver is usable)
  bool ok = false;
  std::string error;
};

Smi g_smi;
std::mutex g_smi_mu;       // amd-smi calls are serialised process-wide
bool g_smi_tried = false;

uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

template <typename T>
bool sym(void* lib, const char* name, T& out) {
  out = reinterpret_cast<T>(dlsym(lib, name));
  return out != nullptr;
}

int smi_open() {
  std::lock_guard<std::mutex> g(g_smi_mu);
  if (g_smi_tried) return g_smi.ok ? int(g_smi.gpus.size()) : -1;
  g_smi_tried = true;
  const char* names[] = {"libamd_smi.so", "/opt/rocm/lib/libamd_smi.so", "libamd_smi.so.26"};
  for (const char* n : names) {
    g_smi.lib = dlopen(n, RTLD_NOW | RTLD_LOCAL);
    if (g_smi.lib) break;
  }
  if (!g_smi.lib) {
    g_smi.error = "libamd_smi.so not found";
    return -1;
  }
  bool ok = sym(g_smi.lib, "amdsmi_init", g_smi.init) && sym(g_smi.lib, "amdsmi_shut_down", g_smi.shutdown) &&
            sym(g_smi.lib, "amdsmi_get_socket_handles", g_smi.sockets) &&
            sym(g_smi.lib, "amdsmi_get_processor_handles", g_smi.procs) &&
            sym(g_smi.lib, "amdsmi_get_energy_count", g_smi.energy);
  sym(g_smi.lib, "amdsmi_get_power_info", g_smi.power);
  sym(g_smi.lib, "amdsmi_get_gpu_activity", g_smi.activity);
  sym(g_smi.lib, "amdsmi_get_gpu_vram_usage", g_smi.vram);
  sym(g_smi.lib, "amdsmi_get_gpu_device_bdf", g_smi.bdf);
  sym(g_smi.lib, "amdsmi_get_processor_type", g_smi.ptype);
  if (!ok) {
    g_smi.error = "libamd_smi.so lacks required symbols";
    return -1;
  }
  sym(g_smi.lib, "amdsmi_get_cpu_handles", g_smi.cpu_handles);
  sym(g_smi.lib, "amdsmi_get_cpu_socket_energy", g_smi.cpu_energy);
  // CPU sockets need the HSMP driver (usually root-only on a shared host): try GPUs + CPUs, then GPUs alone.
  // Without a readable /dev/hsmp the CPU init only prints "ESMI Not initialized" and fails: skip it.
  bool cpus_ok = false;
  const bool hsmp = access("/dev/hsmp", R_OK) == 0;
  if (hsmp && g_smi.cpu_handles && g_smi.cpu_energy &&
      g_smi.init(AMDSMI_INIT_AMD_GPUS | AMDSMI_INIT_AMD_CPUS) == AMDSMI_STATUS_SUCCESS) {
    cpus_ok = true;
  } else if (g_smi.init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) {
    g_smi.error = "amdsmi_init failed";
    return -1;
  }
  if (cpus_ok) {
    uint32_t nc = 0;
    if (g_smi.cpu_handles(&nc, nullptr) == AMDSMI_STATUS_SUCCESS && nc > 0) {
      g_smi.cpus.resize(nc);
      if (g_smi.cpu_handles(&nc, g_smi.cpus.data()) != AMDSMI_STATUS_SUCCESS) nc = 0;
      g_smi.cpus.resize(nc);
      uint64_t e = 0;
      for (auto h : g_smi.cpus)
        if (g_smi.cpu_energy(h, &e) != AMDSMI_STATUS_SUCCESS) {
          g_smi.cpus.clear();
          break;
        }
    }
  }
  uint32_t ns = 0;
  if (g_smi.sockets(&ns, nullptr) != AMDSMI_STATUS_SUCCESS) {
    g_smi.error = "amdsmi_get_socket_handles failed";
    return -1;
  }
  std::vector<amdsmi_socket_handle> socks(ns);
  g_smi.sockets(&ns, socks.data());
  for (uint32_t s = 0; s < ns; ++s) {
    uint32_t np = 0;
    if (g_smi.procs(socks[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
    std::vector<amdsmi_processor_handle> ps(np);
    g_smi.procs(socks[s], &np, ps.data());
    for (auto h : ps) {
      if (g_smi.ptype) {
        processor_type_t t;
        if (g_smi.ptype(h, &t) == AMDSMI_STATUS_SUCCESS && t != AMDSMI_PROCESSOR_TYPE_AMD_GPU) continue;
      } else if (!g_smi.cpus.empty()) {
        continue;  // cannot tell GPUs from CPU sockets: keep the CPU path off rather than mix them
      }
      g_smi.gpus.push_back(h);
    }
  }
  g_smi.ok = true;
  return int(g_smi.gpus.size());
}

bool read_energy(int gpu, uint64_t* acc, float* res, uint64_t* ts) {
  if (!g_smi.ok || gpu < 0 || gpu >= int(g_smi.gpus.size())) return false;
  std::lock_guard<std::mutex> g(g_smi_mu);
  return g_smi.energy(g_smi.gpus[gpu], acc, res, ts) == AMDSMI_STATUS_SUCCESS;
}

// ---------------------------------------------------------------- host side
struct CpuTimes {
  uint64_t idle = 0, total = 0;
};

bool read_cpu_times(CpuTimes* out) {
  FILE* f = fopen("/proc/stat", "r");
  if (!f) return false;
  char tag[16];
  unsigned long long v[10] = {0};
  int n = fscanf(f, "%15s %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu", tag, &v[0], &v[1], &v[2], &v[3],
                 &v[4], &v[5], &v[6], &v[7], &v[8], &v[9]);
  fclose(f);
  if (n < 5) return false;
  // user nice system idle iowait irq softirq steal (guest fields are already in user/nice)
  uint64_t idle = v[3] + v[4];
  uint64_t total = 0;
  for (int i = 0; i < 8; ++i) total += v[i];
  out->idle = idle;
  out->total = total;
  return true;
}

double read_mem_percent() {
  FILE* f = fopen("/proc/meminfo", "r");
  if (!f) return NAN;
  char key[64];
  unsigned long long val;
  char unit[16];
  unsigned long long total = 0, avail = 0;
  while (fscanf(f, "%63s %llu %15[^\n]", key, &val, unit) >= 2) {
    if (!strcmp(key, "MemTotal:")) total = val;
    if (!strcmp(key, "MemAvailable:")) avail = val;
    if (total && avail) break;
  }
  fclose(f);
  if (!total) return NAN;
  return 100.0 * double(total - avail) / double(total);
}

bool read_u64_file(const std::string& path, uint64_t* out) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  unsigned long long v = 0;
  const bool ok = fscanf(f, "%llu", &v) == 1;
  fclose(f);
  if (ok) *out = uint64_t(v);
  return ok;
}

std::string read_line_file(const std::string& path) {
  char buf[128] = {0};
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return "";
  if (!fgets(buf, sizeof(buf), f)) buf[0] = 0;
  fclose(f);
  std::string s(buf);
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
  return s;
}

// Increment of a cumulative counter from `last` to `v` with wrap modulus `range` (0: unknown, a backwards step is
// dropped rather than turned into a huge positive one).
uint64_t wrap_delta(uint64_t v, uint64_t last, uint64_t range) {
  if (v >= last) return v - last;
  if (range > last) return (range - last) + v;  // wrapped once
  return 0;
}

// Host CPU energy: a set of cumulative microjoule counters of one kind, summed.  Each counter is accumulated from
// its own deltas with modular wrap handling (RAPL energy_uj wraps at max_energy_range_uj, every few minutes to
// tens of minutes at server package power), so a window that crosses a wrap still integrates correctly.
struct HostCounter {
  std::string path;                    // sysfs file (rapl / hwmon)
  amdsmi_processor_handle h = nullptr;  // amd-smi CPU socket
  uint64_t range = 0;                  // wrap modulus (0: 64-bit, treated as monotone)
  uint64_t last = 0;
  bool have = false;
};

struct HostEnergy {
  std::string source;  // "amdsmi-cpu" | "rapl" | "hwmon" | "" (none: the Python side models it)
  std::vector<HostCounter> ctr;
  double acc_uj = 0;

  bool raw(HostCounter& c, uint64_t* v) {
    if (c.h) {
      std::lock_guard<std::mutex> g(g_smi_mu);
      return g_smi.cpu_energy && g_smi.cpu_energy(c.h, v) == AMDSMI_STATUS_SUCCESS;
    }
    return read_u64_file(c.path, v);
  }

  void open() {
    ctr.clear();
    source.clear();
    if (!g_smi.cpus.empty()) {
      for (auto h : g_smi.cpus) {
        HostCounter c;
        c.h = h;
        ctr.push_back(c);
      }
      source = "amdsmi-cpu";
      return;
    }
    if (DIR* d = opendir("/sys/class/powercap")) {
      while (dirent* e = readdir(d)) {
        std::string n = e->d_name;
        // top-level package zones only: intel-rapl:0, amd-rapl:0 ... (not sub-zones "x:y:z")
        if (n.find("rapl:") == std::string::npos || std::count(n.begin(), n.end(), ':') != 1) continue;
        HostCounter c;
        c.path = "/sys/class/powercap/" + n + "/energy_uj";
        uint64_t v;
        if (access(c.path.c_str(), R_OK) != 0 || !read_u64_file(c.path, &v)) continue;
        read_u64_file("/sys/class/powercap/" + n + "/max_energy_range_uj", &c.range);
        ctr.push_back(c);
      }
      closedir(d);
    }
    if (!ctr.empty()) {
      source = "rapl";
      return;
    }
    if (DIR* d = opendir("/sys/class/hwmon")) {
      while (dirent* e = readdir(d)) {
        std::string base = std::string("/sys/class/hwmon/") + e->d_name;
        if (read_line_file(base + "/name") != "amd_energy") continue;
        for (int i = 1; i < 1024; ++i) {
          std::string lbl = read_line_file(base + "/energy" + std::to_string(i) + "_label");
          if (lbl.empty()) break;
          if (lbl.rfind("Esocket", 0) != 0) continue;
          HostCounter c;
          c.path = base + "/energy" + std::to_string(i) + "_input";
          uint64_t v;
          if (read_u64_file(c.path, &v)) ctr.push_back(c);
        }
      }
      closedir(d);
    }
    if (!ctr.empty()) source = "hwmon";
  }

  // poll every counter; returns the cumulative joules since the first poll (NaN without a source)
  double poll() {
    if (ctr.empty()) return NAN;
    for (auto& c : ctr) {
      uint64_t v = 0;
      if (!raw(c, &v)) continue;
      if (c.have) acc_uj += double(wrap_delta(v, c.last, c.range));
      c.last = v;
      c.have = true;
    }
    return acc_uj * 1e-6;
  }
};

}  // namespace

extern "C" {

struct es_sample_t {
  uint64_t t_ns;       // CLOCK_MONOTONIC
  int32_t gpu;         // sampler-local gpu slot, -1 = host-only sample
  int32_t pad;
  double energy_j;     // cumulative GPU joules since start (NaN if unavailable)
  double power_w;      // instantaneous socket power
  double gfx_pct;      // gfx activity %
  double umc_pct;      // memory-controller activity %
  double vram_pct;     // VRAM used %
  double cpu_pct;      // host CPU utilisation % since previous sample
  double mem_pct;      // host memory used %
  double cpu_energy_j; // cumulative RAPL joules since start (NaN if unavailable)
};

}  // extern "C"

namespace {

struct TracePoint {
  uint64_t host_ns;  // when observed
  uint64_t dev_ns;   // device-side counter timestamp
  double joules;     // cumulative since sampler start
};

struct GpuTrack {
  int smi_index;
  uint64_t last_acc = 0;
  double res_uj = 0;
  bool have = false;
  double joules = 0;
  int64_t best_offset = INT64_MAX;  // min(host_ns - dev_ns)
  std::vector<TracePoint> trace;
};

struct Sampler {
  std::vector<GpuTrack> gpus;
  int period_us = 100000;
  int fast_us = 1000;
  int core = -1;
  std::thread th;
  std::atomic<long> tid{0};  // kernel thread id of the sampling thread (its CPU time is not the client's)
  std::atomic<bool> running{false};
  std::mutex mu;  // guards traces and ring
  std::vector<es_sample_t> ring;
  size_t ring_cap = 1 << 16;
  size_t head = 0, count = 0;  // ring of slow samples
  std::atomic<uint64_t> dropped{0};  // written under mu by the sampler, read lock-free by es_dropped
  uint64_t t_start = 0;
  CpuTimes last_cpu;
  HostEnergy host;
  std::string error;

  void push(const es_sample_t& s) {
    if (ring.size() < ring_cap) ring.resize(ring_cap);
    size_t idx = (head + count) % ring_cap;
    if (count == ring_cap) {  // overwrite oldest
      head = (head + 1) % ring_cap;
      dropped.fetch_add(1, std::memory_order_relaxed);
    } else {
      ++count;
    }
    ring[idx] = s;
  }

  void poll_energy(GpuTrack& g, uint64_t t) {
    uint64_t acc = 0, dev_ts = 0;
    float res = 0;
    if (!read_energy(g.smi_index, &acc, &res, &dev_ts)) return;
    std::lock_guard<std::mutex> l(mu);
    if (!g.have) {
      g.have = true;
      g.last_acc = acc;
      g.res_uj = res;
      g.trace.push_back({t, dev_ts, 0.0});
    } else if (acc != g.last_acc) {
      uint64_t delta = acc >= g.last_acc ? acc - g.last_acc : 0;  // wrap: ignore the step
      g.joules += double(delta) * double(res) * 1e-6;
      g.last_acc = acc;
      g.trace.push_back({t, dev_ts, g.joules});
    }
    int64_t off = int64_t(t) - int64_t(dev_ts);
    if (dev_ts && off < g.best_offset) g.best_offset = off;
  }

  void slow_sample(uint64_t t) {
    CpuTimes c;
    double cpu = NAN;
    if (read_cpu_times(&c)) {
      uint64_t dt = c.total - last_cpu.total, di = c.idle - last_cpu.idle;
      if (last_cpu.total && dt) cpu = 100.0 * double(dt - std::min(di, dt)) / double(dt);
      last_cpu = c;
    }
    double mem = read_mem_percent();
    const double cpu_j = host.poll();
    if (gpus.empty()) {
      es_sample_t s{};
      s.t_ns = t;
      s.gpu = -1;
      s.energy_j = s.power_w = s.gfx_pct = s.umc_pct = s.vram_pct = NAN;
      s.cpu_pct = cpu;
      s.mem_pct = mem;
      s.cpu_energy_j = cpu_j;
      std::lock_guard<std::mutex> l(mu);
      push(s);
      return;
    }
    for (size_t i = 0; i < gpus.size(); ++i) {
      es_sample_t s{};
      s.t_ns = t;
      s.gpu = int32_t(i);
      s.cpu_pct = cpu;
      s.mem_pct = mem;
      s.cpu_energy_j = cpu_j;
      s.power_w = s.gfx_pct = s.umc_pct = s.vram_pct = NAN;
      auto h = g_smi.gpus[gpus[i].smi_index];
      {
        std::lock_guard<std::mutex> g(g_smi_mu);
        amdsmi_power_info_t p;
        if (g_smi.power && g_smi.power(h, &p) == AMDSMI_STATUS_SUCCESS) {
          uint32_t cur = p.current_socket_power;
          s.power_w = (cur != UINT32_MAX && cur != 0) ? double(cur) : double(p.socket_power);
        }
        amdsmi_engine_usage_t a;
        if (g_smi.activity && g_smi.activity(h, &a) == AMDSMI_STATUS_SUCCESS) {
          s.gfx_pct = a.gfx_activity == UINT32_MAX ? NAN : double(a.gfx_activity);
          s.umc_pct = a.umc_activity == UINT32_MAX ? NAN : double(a.umc_activity);
        }
        amdsmi_vram_usage_t v;
        if (g_smi.vram && g_smi.vram(h, &v) == AMDSMI_STATUS_SUCCESS && v.vram_total)
          s.vram_pct = 100.0 * double(v.vram_used) / double(v.vram_total);
      }
      {
        std::lock_guard<std::mutex> l(mu);
        s.energy_j = gpus[i].have ? gpus[i].joules : NAN;
        push(s);
      }
    }
  }

  void pin() {
    cpu_set_t set;
    CPU_ZERO(&set);
    int target = core;
    if (target < 0) {
      cpu_set_t cur;
      CPU_ZERO(&cur);
      if (sched_getaffinity(0, sizeof(cur), &cur) == 0) {
        for (int c = CPU_SETSIZE - 1; c >= 0; --c)
          if (CPU_ISSET(c, &cur)) {
            target = c;
            break;
          }
      }
    }
    if (target >= 0) {
      CPU_SET(target, &set);
      pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    }
  }

  void loop() {
    tid.store(long(syscall(SYS_gettid)), std::memory_order_release);
    pin();
    uint64_t next_slow = now_ns();
    while (running.load(std::memory_order_acquire)) {
      uint64_t t = now_ns();
      for (auto& g : gpus) poll_energy(g, t);
      if (t >= next_slow) {
        slow_sample(t);
        next_slow += uint64_t(period_us) * 1000ull;
        if (next_slow < t) next_slow = t + uint64_t(period_us) * 1000ull;
      }
      timespec req{0, long(fast_us) * 1000L};
      nanosleep(&req, nullptr);
    }
  }

  // cumulative joules of gpu slot at host time t (linear interpolation on the trace)
  double joules_at(const GpuTrack& g, uint64_t t) const {
    const auto& tr = g.trace;
    if (tr.empty()) return NAN;
    auto host_of = [&](const TracePoint& p) -> double {
      // device timestamp mapped to host time when the offset estimate is sane
      if (p.dev_ns && g.best_offset != INT64_MAX) {
        double h = double(int64_t(p.dev_ns) + g.best_offset);
        if (h <= double(p.host_ns) + 1e3 && double(p.host_ns) - h < 50e6) return h;
      }
      return double(p.host_ns);
    };
    double tt = double(t);
    if (tt <= host_of(tr.front())) return tr.front().joules;
    if (tt >= host_of(tr.back())) {
      // extrapolate with the last segment's slope (bounded to one counter interval)
      if (tr.size() < 2) return tr.back().joules;
      const auto& a = tr[tr.size() - 2];
      const auto& b = tr.back();
      double ha = host_of(a), hb = host_of(b);
      if (hb <= ha) return b.joules;
      double slope = (b.joules - a.joules) / (hb - ha);
      double span = std::min(tt - hb, hb - ha);
      return b.joules + slope * span;
    }
    size_t lo = 0, hi = tr.size() - 1;
    while (hi - lo > 1) {
      size_t mid = (lo + hi) / 2;
      if (host_of(tr[mid]) <= tt)
        lo = mid;
      else
        hi = mid;
    }
    double ha = host_of(tr[lo]), hb = host_of(tr[hi]);
    if (hb <= ha) return tr[hi].joules;
    double f = (tt - ha) / (hb - ha);
    // energy reported at point hi accrued over (ha, hb]
    return tr[lo].joules + f * (tr[hi].joules - tr[lo].joules);
  }
};

}  // namespace

extern "C" {

int es_init(void) { return smi_open(); }

const char* es_last_error(void) { return g_smi.error.c_str(); }

int es_gpu_count(void) { return g_smi.ok ? int(g_smi.gpus.size()) : 0; }

int es_gpu_bdf(int idx, uint32_t* domain, uint32_t* bus, uint32_t* device, uint32_t* function) {
  if (!g_smi.ok || !g_smi.bdf || idx < 0 || idx >= int(g_smi.gpus.size())) return -1;
  amdsmi_bdf_t b;
  std::lock_guard<std::mutex> g(g_smi_mu);
  if (g_smi.bdf(g_smi.gpus[idx], &b) != AMDSMI_STATUS_SUCCESS) return -1;
  *domain = uint32_t(b.domain_number);
  *bus = uint32_t(b.bus_number);
  *device = uint32_t(b.device_number);
  *function = uint32_t(b.function_number);
  return 0;
}

int es_read_energy(int idx, uint64_t* acc, float* res, uint64_t* ts) {
  return read_energy(idx, acc, res, ts) ? 0 : -1;
}

uint64_t es_now_ns(void) { return now_ns(); }

void* es_create(const int* gpu_idx, int n, int period_us, int fast_period_us, int cpu_core, int ring_cap) {
  smi_open();
  auto* s = new Sampler();
  for (int i = 0; i < n; ++i) {
    if (gpu_idx[i] < 0 || gpu_idx[i] >= es_gpu_count()) continue;
    GpuTrack g;
    g.smi_index = gpu_idx[i];
    s->gpus.push_back(std::move(g));
  }
  s->period_us = std::max(1000, period_us);
  s->fast_us = std::max(200, fast_period_us);
  s->core = cpu_core;
  if (ring_cap > 0) s->ring_cap = size_t(ring_cap);
  s->host.open();
  return s;
}

int es_num_tracked(void* h) { return h ? int(static_cast<Sampler*>(h)->gpus.size()) : 0; }

int es_start(void* h) {
  auto* s = static_cast<Sampler*>(h);
  if (!s || s->running.load()) return -1;
  s->t_start = now_ns();
  read_cpu_times(&s->last_cpu);
  s->host.poll();  // first reading: the zero of the cumulative host joules
  for (auto& g : s->gpus) s->poll_energy(g, s->t_start);
  s->running.store(true, std::memory_order_release);
  s->th = std::thread([s] { s->loop(); });
  return 0;
}

int es_stop(void* h) {
  auto* s = static_cast<Sampler*>(h);
  if (!s || !s->running.load()) return -1;
  s->running.store(false, std::memory_order_release);
  if (s->th.joinable()) s->th.join();
  uint64_t t = now_ns();
  for (auto& g : s->gpus) s->poll_energy(g, t);
  return 0;
}

void es_destroy(void* h) {
  auto* s = static_cast<Sampler*>(h);
  if (!s) return;
  if (s->running.load()) es_stop(h);
  delete s;
}

// Energy (J) of tracked gpu slot between two CLOCK_MONOTONIC instants.
double es_energy_between(void* h, int slot, uint64_t t0, uint64_t t1) {
  auto* s = static_cast<Sampler*>(h);
  if (!s || slot < 0 || slot >= int(s->gpus.size())) return NAN;
  std::lock_guard<std::mutex> l(s->mu);
  const auto& g = s->gpus[slot];
  return s->joules_at(g, t1) - s->joules_at(g, t0);
}

// Number of counter updates seen for a slot (diagnostics: cadence).
int64_t es_trace_points(void* h, int slot) {
  auto* s = static_cast<Sampler*>(h);
  if (!s || slot < 0 || slot >= int(s->gpus.size())) return -1;
  std::lock_guard<std::mutex> l(s->mu);
  return int64_t(s->gpus[slot].trace.size());
}

// Copy up to max trace points (host_ns, joules) of a slot; returns count.
int es_trace(void* h, int slot, uint64_t* t_out, double* j_out, int max) {
  auto* s = static_cast<Sampler*>(h);
  if (!s || slot < 0 || slot >= int(s->gpus.size())) return -1;
  std::lock_guard<std::mutex> l(s->mu);
  const auto& tr = s->gpus[slot].trace;
  int n = std::min<int>(max, int(tr.size()));
  size_t off = tr.size() - size_t(n);
  for (int i = 0; i < n; ++i) {
    t_out[i] = tr[off + i].host_ns;
    j_out[i] = tr[off + i].joules;
  }
  return n;
}

// Drop trace points older than t (keeps one point before t for interpolation).
void es_trim(void* h, uint64_t t) {
  auto* s = static_cast<Sampler*>(h);
  if (!s) return;
  std::lock_guard<std::mutex> l(s->mu);
  for (auto& g : s->gpus) {
    auto& tr = g.trace;
    size_t k = 0;
    while (k + 1 < tr.size() && tr[k + 1].host_ns < t) ++k;
    if (k) tr.erase(tr.begin(), tr.begin() + long(k));
  }
}

// Drain slow samples into out (oldest first); returns count.
int es_drain(void* h, es_sample_t* out, int max) {
  auto* s = static_cast<Sampler*>(h);
  if (!s) return -1;
  std::lock_guard<std::mutex> l(s->mu);
  int n = 0;
  while (s->count && n < max) {
    out[n++] = s->ring[s->head];
    s->head = (s->head + 1) % s->ring_cap;
    --s->count;
  }
  return n;
}

uint64_t es_dropped(void* h) { return h ? static_cast<Sampler*>(h)->dropped.load(std::memory_order_relaxed) : 0; }

int es_sample_size(void) { return int(sizeof(es_sample_t)); }

// Kernel thread id of the running sampler thread (0 before es_start): process-attributed CPU energy leaves the
// measurement's own thread out of the client's CPU time (cain_amd/energy/meter.py).
long es_sampler_tid(void* h) { return h ? static_cast<Sampler*>(h)->tid.load(std::memory_order_acquire) : 0; }

// Host CPU energy source of a sampler: "amdsmi-cpu", "rapl", "hwmon" or "" (none readable).
const char* es_host_energy_source(void* h) { return h ? static_cast<Sampler*>(h)->host.source.c_str() : ""; }

// Test hook: feed raw readings of one counter with modulus `range` through the wrap-aware accumulator; returns
// the accumulated joules (tests/test_energy.py).
double es_test_wrap_accumulate(const uint64_t* raw, int n, uint64_t range) {
  double acc = 0;
  uint64_t last = 0;
  for (int i = 0; i < n; ++i) {
    if (i) acc += double(wrap_delta(raw[i], last, range));
    last = raw[i];
  }
  return acc * 1e-6;
}

}  // extern "C"
