// sn_loader — native minibatch pipeline: record sources -> sampler -> worker threads ->
// ring of pinned host slots -> hipMemcpyAsync on the caller's copy stream.
//
// Replaces, natively, what the reference splits across the JVM and Caffe:
//   * SparkNet's per-round minibatch selection (src/main/scala/libs/MinibatchSampler.scala:
//     18-58: a random contiguous window of tau minibatches per round) and the CIFAR binary
//     ingest (src/main/scala/loaders/CifarLoader.scala:15-85);
//   * Caffe's prefetching data path: BasePrefetchingDataLayer's PREFETCH_COUNT=3 batches,
//     InternalThread + BlockingQueue + async_gpu_push on a side stream
//     (caffe/src/caffe/layers/base_data_layer.cpp:70-96, caffe/src/caffe/util/
//     blocking_queue.cpp) and the per-sample DataReader cursor (data_reader.cpp).
// Design (MI355X host side): N worker threads fill whole batches in parallel (batch b's
// sample list is a pure function of (seed, b), so workers never coordinate beyond slot
// ownership); slots are hipHostMalloc'd so the H2D copy runs at full PCIe/xGMI rate on a
// side stream; a slot is refilled only after the hipEvent recorded behind its copy has
// completed.  No Python on the data path; the training thread only calls acquire/copy.
#include <hip/hip_runtime_api.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

extern "C" {

struct SnLoaderConfig {
  int source;  // 0 = fixed-size record files (CIFAR-10/100 binary), 1 = host arrays, 2 = synthetic
  const char* paths;  // '\n'-separated file list (source 0)
  long long header_bytes;  // bytes skipped at the start of every file
  long long record_bytes;  // bytes per record (source 0)
  long long label_offset, label_bytes;  // label field inside a record (little-endian, 1/2/4 bytes)
  long long image_offset;  // image field inside a record
  const uint8_t* mem_images;  // source 1: [count][image_bytes]
  const int32_t* mem_labels;  // source 1: [count]
  long long mem_count;
  long long image_bytes;  // C*H*W bytes per sample
  int batch;
  int sampler;  // 0 = per-epoch shuffle, 1 = sequential (wraps), 2 = SparkNet window of tau
  int tau;
  int rank, world;  // contiguous shard of the records
  unsigned long long seed;
  int slots, threads;
  int pinned;  // 1: hipHostMalloc the ring (GPU hosts), 0: plain aligned host memory
  int classes;  // synthetic labels
  long long synthetic_count;  // synthetic: samples in the (virtual) dataset
  long long first_batch;  // sequence number of the first batch delivered (resume mid-stream)
};

struct SnLoaderStats {
  long long batches_filled, batches_consumed;
  double fill_seconds, consumer_wait_seconds;
  long long shard_samples, batches_per_epoch;
};

}  // extern "C"

namespace {

enum SlotState { FREE = 0, FILLING = 1, READY = 2, HANDED = 3 };

struct Slot {
  uint8_t* img = nullptr;
  int32_t* lab = nullptr;
  int state = FREE;
  long long seq = -1;        // batch sequence number stored / expected in this slot
  hipEvent_t ev = nullptr;   // recorded after the H2D copy of this slot
  bool ev_pending = false;
};

struct MappedFile {
  const uint8_t* base = nullptr;
  size_t size = 0;
};

inline uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

class Loader {
 public:
  explicit Loader(const SnLoaderConfig& c) : cfg_(c) {}
  ~Loader() { shutdown(); }

  int init() {
    if (cfg_.batch <= 0 || cfg_.image_bytes <= 0 || cfg_.slots < 2 || cfg_.threads < 1) return 1;
    if (cfg_.world < 1 || cfg_.rank < 0 || cfg_.rank >= cfg_.world) return 2;
    if (cfg_.sampler == 2 && cfg_.tau < 1) return 3;
    long long total = 0;
    if (cfg_.source == 0) {
      if (int rc = map_files(&total)) return rc;
    } else if (cfg_.source == 1) {
      if (!cfg_.mem_images || !cfg_.mem_labels) return 4;
      total = cfg_.mem_count;
    } else if (cfg_.source == 2) {
      total = cfg_.synthetic_count > 0 ? cfg_.synthetic_count : (long long)cfg_.batch * cfg_.slots;
    } else {
      return 5;
    }
    // contiguous deterministic shard (sampler.shard_range)
    const long long per = total / cfg_.world, rem = total % cfg_.world;
    shard_lo_ = cfg_.rank * per + std::min<long long>(cfg_.rank, rem);
    shard_n_ = per + (cfg_.rank < rem ? 1 : 0);
    batches_per_epoch_ = shard_n_ / cfg_.batch;  // the remainder is dropped (ScaleAndConvert.scala:45-70)
    if (batches_per_epoch_ < 1) return 6;
    if (cfg_.sampler == 2 && cfg_.tau > batches_per_epoch_) return 7;
    slots_.resize(cfg_.slots);
    const size_t ibytes = (size_t)cfg_.batch * cfg_.image_bytes, lbytes = (size_t)cfg_.batch * sizeof(int32_t);
    for (auto& s : slots_) {
      if (cfg_.pinned) {
        if (hipHostMalloc((void**)&s.img, ibytes, hipHostMallocDefault) != hipSuccess) return 8;
        if (hipHostMalloc((void**)&s.lab, lbytes, hipHostMallocDefault) != hipSuccess) return 8;
        if (hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) return 9;
      } else {
        s.img = static_cast<uint8_t*>(std::aligned_alloc(4096, (ibytes + 4095) / 4096 * 4096));
        s.lab = static_cast<int32_t*>(std::aligned_alloc(64, (lbytes + 63) / 64 * 64));
        if (!s.img || !s.lab) return 8;
      }
    }
    if (cfg_.first_batch < 0) return 1;
    next_fill_ = cfg_.first_batch;
    next_consume_ = cfg_.first_batch;
    for (int i = 0; i < cfg_.slots; ++i) {  // slot (b % slots) first holds batch b
      const long long b = cfg_.first_batch + i;
      slots_[b % cfg_.slots].seq = b;
    }
    for (int t = 0; t < cfg_.threads; ++t) workers_.emplace_back([this] { worker(); });
    return 0;
  }

  // Blocks until batch `next_consume_` is ready; returns its sequence number.
  long long acquire(uint8_t** img, int32_t** lab) {
    const long long b = next_consume_++;
    Slot& s = slots_[b % cfg_.slots];
    auto t0 = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(mu_);
    cv_ready_.wait(lk, [&] { return stop_ || (s.seq == b && s.state == READY); });
    if (stop_) return -1;
    s.state = HANDED;
    wait_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    ++consumed_;
    *img = s.img;
    *lab = s.lab;
    return b;
  }

  int copy_async(long long b, void* dev_img, void* dev_lab, hipStream_t st) {
    Slot& s = slots_[b % cfg_.slots];
    if (s.seq != b || s.state != HANDED) return 10;
    const size_t ibytes = (size_t)cfg_.batch * cfg_.image_bytes, lbytes = (size_t)cfg_.batch * sizeof(int32_t);
    if (hipMemcpyAsync(dev_img, s.img, ibytes, hipMemcpyHostToDevice, st) != hipSuccess) return 11;
    if (hipMemcpyAsync(dev_lab, s.lab, lbytes, hipMemcpyHostToDevice, st) != hipSuccess) return 11;
    if (s.ev) {
      if (hipEventRecord(s.ev, st) != hipSuccess) return 12;
      s.ev_pending = true;
    }
    return 0;
  }

  // The slot may be refilled with batch b + slots (after its copy event completes).
  int release(long long b) {
    Slot& s = slots_[b % cfg_.slots];
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (s.seq != b || s.state != HANDED) return 13;
      s.state = FREE;
      s.seq = b + cfg_.slots;
    }
    cv_free_.notify_all();
    return 0;
  }

  void stats(SnLoaderStats* out) {
    std::lock_guard<std::mutex> lk(mu_);
    out->batches_filled = filled_;
    out->batches_consumed = consumed_;
    out->fill_seconds = fill_s_;
    out->consumer_wait_seconds = wait_s_;
    out->shard_samples = shard_n_;
    out->batches_per_epoch = batches_per_epoch_;
  }

  // Sample indices (shard-relative) of batch b — exposed for tests / reproducibility.
  void batch_indices(long long b, long long* out) {
    std::vector<long long> v;
    indices(b, v);
    std::copy(v.begin(), v.end(), out);
  }

  void shutdown() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_free_.notify_all();
    cv_ready_.notify_all();
    for (auto& t : workers_)
      if (t.joinable()) t.join();
    workers_.clear();
    for (auto& s : slots_) {
      if (cfg_.pinned) {
        if (s.ev) {
          (void)hipEventSynchronize(s.ev);
          (void)hipEventDestroy(s.ev);
        }
        if (s.img) (void)hipHostFree(s.img);
        if (s.lab) (void)hipHostFree(s.lab);
      } else {
        std::free(s.img);
        std::free(s.lab);
      }
      s.img = nullptr;
      s.lab = nullptr;
      s.ev = nullptr;
    }
    slots_.clear();
    for (auto& f : files_)
      if (f.base) munmap(const_cast<uint8_t*>(f.base), f.size);
    files_.clear();
  }

 private:
  int map_files(long long* total) {
    if (!cfg_.paths || cfg_.record_bytes <= 0) return 4;
    if (cfg_.label_bytes != 1 && cfg_.label_bytes != 2 && cfg_.label_bytes != 4) return 4;
    if (cfg_.image_offset + cfg_.image_bytes > cfg_.record_bytes) return 4;
    std::string all(cfg_.paths);
    size_t pos = 0;
    while (pos <= all.size()) {
      size_t nl = all.find('\n', pos);
      std::string p = all.substr(pos, nl == std::string::npos ? std::string::npos : nl - pos);
      pos = nl == std::string::npos ? all.size() + 1 : nl + 1;
      if (p.empty()) continue;
      int fd = open(p.c_str(), O_RDONLY);
      if (fd < 0) return 20;
      struct stat st;
      if (fstat(fd, &st) != 0) {
        close(fd);
        return 20;
      }
      MappedFile mf;
      mf.size = (size_t)st.st_size;
      void* m = mmap(nullptr, mf.size, PROT_READ, MAP_PRIVATE, fd, 0);
      close(fd);
      if (m == MAP_FAILED) return 21;
      madvise(m, mf.size, MADV_WILLNEED);
      mf.base = static_cast<const uint8_t*>(m);
      const long long n = ((long long)mf.size - cfg_.header_bytes) / cfg_.record_bytes;
      file_first_.push_back(*total);
      *total += std::max(0ll, n);
      files_.push_back(mf);
    }
    return files_.empty() ? 20 : 0;
  }

  // Shared ownership: a worker keeps its epoch's permutation alive while it reads it,
  // even if other workers have since evicted that epoch from the small cache.
  std::shared_ptr<const std::vector<long long>> perm(long long epoch) {
    std::lock_guard<std::mutex> lk(perm_mu_);
    auto it = perms_.find(epoch);
    if (it != perms_.end()) return it->second;
    auto p = std::make_shared<std::vector<long long>>(shard_n_);
    for (long long i = 0; i < shard_n_; ++i) (*p)[i] = i;
    std::mt19937_64 g(splitmix(cfg_.seed ^ splitmix((uint64_t)epoch + 1)));
    for (long long i = shard_n_ - 1; i > 0; --i) {
      long long j = (long long)(g() % (uint64_t)(i + 1));
      std::swap((*p)[i], (*p)[j]);
    }
    if (perms_.size() > 3) perms_.erase(perms_.begin());
    perms_.emplace(epoch, p);
    return p;
  }

  void indices(long long b, std::vector<long long>& out) {
    out.resize(cfg_.batch);
    const long long P = batches_per_epoch_;
    if (cfg_.sampler == 0) {
      const auto p = perm(b / P);
      const long long k = b % P;
      for (int i = 0; i < cfg_.batch; ++i) out[i] = (*p)[k * cfg_.batch + i];
    } else if (cfg_.sampler == 1) {
      for (int i = 0; i < cfg_.batch; ++i) out[i] = (b * cfg_.batch + i) % shard_n_;
    } else {
      // SparkNet MinibatchSampler: round r = b / tau starts at a uniform window in [0, P - tau]
      const long long r = b / cfg_.tau, j = b % cfg_.tau;
      std::mt19937_64 g(splitmix(cfg_.seed * 0x2545F4914F6CDD1Dull + (uint64_t)r));
      const long long start = (long long)(g() % (uint64_t)(P - cfg_.tau + 1));
      const long long m = start + j;
      for (int i = 0; i < cfg_.batch; ++i) out[i] = m * cfg_.batch + i;
    }
  }

  void fill(long long b, Slot& s) {
    std::vector<long long> idx;
    indices(b, idx);
    const long long ib = cfg_.image_bytes;
    for (int i = 0; i < cfg_.batch; ++i) {
      const long long gi = shard_lo_ + idx[i];  // global record index
      uint8_t* dst = s.img + (size_t)i * ib;
      if (cfg_.source == 0) {
        size_t f = std::upper_bound(file_first_.begin(), file_first_.end(), gi) - file_first_.begin() - 1;
        const uint8_t* rec = files_[f].base + cfg_.header_bytes + (gi - file_first_[f]) * cfg_.record_bytes;
        std::memcpy(dst, rec + cfg_.image_offset, (size_t)ib);
        uint32_t lab = 0;
        std::memcpy(&lab, rec + cfg_.label_offset, (size_t)cfg_.label_bytes);
        s.lab[i] = (int32_t)lab;
      } else if (cfg_.source == 1) {
        std::memcpy(dst, cfg_.mem_images + (size_t)gi * ib, (size_t)ib);
        s.lab[i] = cfg_.mem_labels[gi];
      } else {
        uint64_t x = splitmix(cfg_.seed ^ splitmix((uint64_t)gi));
        long long k = 0;
        for (; k + 8 <= ib; k += 8) {
          x ^= x << 13;
          x ^= x >> 7;
          x ^= x << 17;
          std::memcpy(dst + k, &x, 8);
        }
        for (; k < ib; ++k) dst[k] = (uint8_t)(x >> (8 * (k & 7)));
        s.lab[i] = (int32_t)(splitmix((uint64_t)gi * 31 + cfg_.seed) % (uint64_t)std::max(1, cfg_.classes));
      }
    }
  }

  void worker() {
    for (;;) {
      const long long b = next_fill_.fetch_add(1);
      Slot& s = slots_[b % cfg_.slots];
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_free_.wait(lk, [&] { return stop_ || (s.seq == b && s.state == FREE); });
        if (stop_) return;
        s.state = FILLING;
      }
      if (s.ev && s.ev_pending) {  // the previous occupant's H2D copy must have landed
        (void)hipEventSynchronize(s.ev);
        s.ev_pending = false;
      }
      auto t0 = std::chrono::steady_clock::now();
      fill(b, s);
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      {
        std::lock_guard<std::mutex> lk(mu_);
        s.state = READY;
        ++filled_;
        fill_s_ += dt;
      }
      cv_ready_.notify_all();
    }
  }

  SnLoaderConfig cfg_;
  std::vector<MappedFile> files_;
  std::vector<long long> file_first_;
  long long shard_lo_ = 0, shard_n_ = 0, batches_per_epoch_ = 0;
  std::vector<Slot> slots_;
  std::vector<std::thread> workers_;
  std::mutex mu_, perm_mu_;
  std::condition_variable cv_free_, cv_ready_;
  std::atomic<long long> next_fill_{0};
  long long next_consume_ = 0;
  bool stop_ = false;
  std::map<long long, std::shared_ptr<const std::vector<long long>>> perms_;
  long long filled_ = 0, consumed_ = 0;
  double fill_s_ = 0.0, wait_s_ = 0.0;
};

}  // namespace

extern "C" {

void* sn_loader_create(const SnLoaderConfig* cfg, int* err) {
  auto* L = new Loader(*cfg);
  int rc = L->init();
  if (err) *err = rc;
  if (rc != 0) {
    delete L;
    return nullptr;
  }
  return L;
}

long long sn_loader_acquire(void* h, uint8_t** img, int32_t** lab) {
  return static_cast<Loader*>(h)->acquire(img, lab);
}

int sn_loader_copy_async(void* h, long long seq, void* dev_img, void* dev_lab, hipStream_t stream) {
  return static_cast<Loader*>(h)->copy_async(seq, dev_img, dev_lab, stream);
}

int sn_loader_release(void* h, long long seq) { return static_cast<Loader*>(h)->release(seq); }

void sn_loader_stats(void* h, SnLoaderStats* out) { static_cast<Loader*>(h)->stats(out); }

void sn_loader_batch_indices(void* h, long long seq, long long* out) {
  static_cast<Loader*>(h)->batch_indices(seq, out);
}

void sn_loader_destroy(void* h) { delete static_cast<Loader*>(h); }

}  // extern "C"
