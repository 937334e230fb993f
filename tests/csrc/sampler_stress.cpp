// Host-side concurrency stress of the energy sampler (cain_amd/energy/csrc/sampler.cpp), built by
// tests/test_sanitizers.py with -fsanitize=thread and with -fsanitize=address,undefined.
// No GPU is needed: without amd-smi the sampler still runs its host-metric thread (CPU %, memory %,
// RAPL), which is exactly the producer/consumer path the Python meter drains.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <vector>

extern "C" {
struct es_sample_t {
  uint64_t t_ns;
  int32_t gpu, pad;
  double energy_j, power_w, gfx_pct, umc_pct, vram_pct, cpu_pct, mem_pct, cpu_energy_j;
};
int es_init(void);
void* es_create(const int* gpu_idx, int n, int period_us, int fast_period_us, int cpu_core, int ring_cap);
int es_start(void* h);
int es_stop(void* h);
void es_destroy(void* h);
int es_drain(void* h, es_sample_t* out, int max);
uint64_t es_dropped(void* h);
int64_t es_trace_points(void* h, int slot);
uint64_t es_now_ns(void);
int es_sample_size(void);
}

int main() {
  if (es_sample_size() != int(sizeof(es_sample_t))) return 2;
  es_init();
  long drained = 0;
  for (int cycle = 0; cycle < 4; ++cycle) {
    void* h = es_create(nullptr, 0, /*period_us=*/500, /*fast_period_us=*/200, /*cpu_core=*/-1, /*ring_cap=*/16);
    if (!h || es_start(h) != 0) return 3;
    std::atomic<bool> stop{false};
    std::vector<std::thread> readers;
    std::atomic<long> got{0};
    const bool lazy = cycle % 2 == 1;  // odd cycles: let the ring overflow so drops are counted
    readers.emplace_back([&] {
      es_sample_t buf[8];
      while (!stop.load()) {
        if (lazy) std::this_thread::sleep_for(std::chrono::milliseconds(20));
        got += es_drain(h, buf, lazy ? 1 : 8);
      }
    });
    readers.emplace_back([&] {
      uint64_t last = 0;
      while (!stop.load()) {
        last += es_dropped(h);
        (void)es_trace_points(h, 0);
        (void)es_now_ns();
      }
      (void)last;
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(60));
    stop = true;
    for (auto& t : readers) t.join();
    es_stop(h);
    es_sample_t buf[64];
    got += es_drain(h, buf, 64);
    if (lazy && es_dropped(h) == 0) return 5;  // the overflow path must have run
    es_destroy(h);
    drained += got.load();
  }
  std::printf("drained %ld samples\n", drained);
  return drained > 0 ? 0 : 4;
}
