// Host-only stress driver for csrc/runtime/loader.cpp, built under ThreadSanitizer and
// AddressSanitizer+UBSan by tests/test_native_sanitizers.py (sanitizer builds
// of the host library; the ring / worker protocol is the concurrency-heavy part).
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

extern "C" {
struct SnLoaderConfig {
  int source;
  const char* paths;
  long long header_bytes, record_bytes, label_offset, label_bytes, image_offset;
  const uint8_t* mem_images;
  const int32_t* mem_labels;
  long long mem_count;
  long long image_bytes;
  int batch, sampler, tau, rank, world;
  unsigned long long seed;
  int slots, threads, pinned, classes;
  long long synthetic_count, first_batch;
};
void* sn_loader_create(const SnLoaderConfig*, int*);
long long sn_loader_acquire(void*, uint8_t**, int32_t**);
int sn_loader_release(void*, long long);
void sn_loader_batch_indices(void*, long long, long long*);
void sn_loader_destroy(void*);
}

int main() {
  const int n = 997, ib = 3 * 8 * 8, B = 16;
  std::vector<uint8_t> imgs((size_t)n * ib);
  std::vector<int32_t> labs(n);
  std::mt19937 g(1);
  for (auto& v : imgs) v = (uint8_t)g();
  for (int i = 0; i < n; ++i) labs[i] = i;
  int bad = 0;
  for (int sampler = 0; sampler < 3; ++sampler) {
    for (int threads : {1, 3, 8}) {
      SnLoaderConfig c;
      std::memset(&c, 0, sizeof(c));
      c.source = 1;
      c.mem_images = imgs.data();
      c.mem_labels = labs.data();
      c.mem_count = n;
      c.image_bytes = ib;
      c.batch = B;
      c.sampler = sampler;
      c.tau = 5;
      c.world = 1;
      c.seed = 7;
      c.slots = 3;
      c.threads = threads;
      c.first_batch = sampler == 2 ? 11 : 0;
      int err = 0;
      void* h = sn_loader_create(&c, &err);
      if (!h) { std::printf("create failed %d\n", err); return 2; }
      std::vector<long long> idx(B);
      for (int it = 0; it < 60; ++it) {
        uint8_t* im;
        int32_t* lb;
        long long seq = sn_loader_acquire(h, &im, &lb);
        sn_loader_batch_indices(h, seq, idx.data());
        for (int i = 0; i < B; ++i) {
          if (lb[i] != labs[idx[i]] || std::memcmp(im + (size_t)i * ib, &imgs[(size_t)idx[i] * ib], ib)) ++bad;
        }
        if (it % 7 == 0) std::this_thread::sleep_for(std::chrono::microseconds(200));
        sn_loader_release(h, seq);
      }
      sn_loader_destroy(h);  // workers still blocked on slots must be joined cleanly
    }
  }
  // Many epochs in flight at once (1 batch per epoch, 8 slots, 8 threads): workers read
  // permutations that other workers evict from the loader's epoch cache.
  {
    SnLoaderConfig c;
    std::memset(&c, 0, sizeof(c));
    c.source = 1;
    c.mem_images = imgs.data();
    c.mem_labels = labs.data();
    c.mem_count = B;
    c.image_bytes = ib;
    c.batch = B;
    c.sampler = 0;
    c.world = 1;
    c.seed = 3;
    c.slots = 8;
    c.threads = 8;
    int err = 0;
    void* h = sn_loader_create(&c, &err);
    if (!h) { std::printf("create failed %d\n", err); return 2; }
    std::vector<long long> idx(B);
    for (int it = 0; it < 400; ++it) {
      uint8_t* im;
      int32_t* lb;
      long long seq = sn_loader_acquire(h, &im, &lb);
      sn_loader_batch_indices(h, seq, idx.data());
      for (int i = 0; i < B; ++i)
        if (lb[i] != labs[idx[i]] || std::memcmp(im + (size_t)i * ib, &imgs[(size_t)idx[i] * ib], ib)) ++bad;
      sn_loader_release(h, seq);
    }
    sn_loader_destroy(h);
  }
  std::printf("bad=%d\n", bad);
  return bad ? 1 : 0;
}
