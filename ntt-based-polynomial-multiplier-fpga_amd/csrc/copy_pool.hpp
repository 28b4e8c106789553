// copy_pool.hpp — the host-buffer path's staging memcpy split over a few host threads
// (csrc/nttmul.cpp pcopy).  Header-only and free of HIP so that tests/sanitize/tsan_copy_pool.cpp
// can drive it under ThreadSanitizer (tests/test_sanitizers.py).
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

namespace nttmul {

// memcpy split over a few host threads for large blocks (the staging copies bound the
// host-buffer path: one core moves ~10-20 GB/s, a PCIe Gen5 x16 link ~50 GB/s each way).  The
// workers are started once and live for the process (never joined: the pool is never freed).
//
// Concurrent calls share the pool instead of queueing behind each other (verdict r5 item 3: a
// multi-device context drives one host thread per device slice, and each slice's staging copies
// are its own PCIe link's traffic, NTT_PCIECommunicationv2.c:171-224 per board).  A call posts a
// job of `parts` equal pieces; idle workers take pieces of whichever jobs are posted, in posting
// order, and the calling thread works through its own job's pieces as well, so a call always
// finishes even while every worker is busy with other callers' jobs.
constexpr unsigned kMaxCopyThreads = 64;
class CopyPool {
 public:
  static CopyPool &get() {
    static CopyPool *pool = new CopyPool();
    return *pool;
  }
  // split over at most `threads` threads (the caller's included)
  void copy(void *dst, const void *src, size_t bytes, unsigned threads) {
    const size_t kPart = 1u << 20;
    size_t parts = std::min<size_t>(std::min<size_t>(cap_, threads), bytes / kPart);
    if (parts > 1) {
      std::lock_guard<std::mutex> l(mu_);
      parts = std::min<size_t>(parts, grow((unsigned)parts - 1) + 1);
    }
    if (parts <= 1) {
      memcpy(dst, src, bytes);
      return;
    }
    // ceiling split (advisor r5: a floor step left bytes % parts uncopied whenever bytes / parts
    // was a multiple of 4 KiB), rounded up to whole 4 KiB pages; then as many pieces as it takes
    const size_t step = ((bytes + parts - 1) / parts + 4095) & ~(size_t)4095;
    Job job;
    job.d = (char *)dst;
    job.s = (const char *)src;
    job.bytes = bytes;
    job.step = step;
    job.parts = (unsigned)((bytes + step - 1) / step);
    job.left = job.parts;
    const unsigned now = inflight_.fetch_add(1) + 1;
    for (unsigned m = max_inflight_.load(); now > m && !max_inflight_.compare_exchange_weak(m, now);) {
    }
    std::unique_lock<std::mutex> l(mu_);
    jobs_.push_back(&job);
    for (unsigned i = 1; i < job.parts; i++) work_.notify_one();
    while (job.next < job.parts) {  // the caller's share: whatever pieces no worker has taken
      const unsigned p = claim(job);
      l.unlock();
      piece(job, p);
      l.lock();
      --job.left;
    }
    job.done.wait(l, [&] { return job.left == 0; });
    l.unlock();
    inflight_.fetch_sub(1);
  }
  // instrumentation (tests/sanitize/tsan_copy_pool.cpp): the most split copies seen in flight
  // at once, and the worker threads running
  unsigned max_concurrent_splits() const { return max_inflight_.load(); }
  unsigned workers() {
    std::lock_guard<std::mutex> l(mu_);
    return started_;
  }

 private:
  struct Job {
    char *d = nullptr;
    const char *s = nullptr;
    size_t bytes = 0, step = 0;
    unsigned parts = 0, next = 0, left = 0;  // next, left: guarded by mu_
    std::condition_variable done;
  };
  CopyPool() {
    const unsigned hw = std::thread::hardware_concurrency();
    cap_ = std::min(kMaxCopyThreads, std::max(hw, 1u));
  }
  // the next unclaimed piece of `j` (mu_ held); a job leaves the queue with its last piece
  unsigned claim(Job &j) {
    const unsigned p = j.next++;
    if (j.next == j.parts) jobs_.erase(std::find(jobs_.begin(), jobs_.end(), &j));
    return p;
  }
  static void piece(const Job &j, unsigned p) {
    const size_t o = (size_t)p * j.step;
    if (o < j.bytes) memcpy(j.d + o, j.s + o, std::min(j.step, j.bytes - o));
  }
  // Workers start on first use, up to the largest split any context has asked for (advisor r4:
  // not min(64, hardware threads) - 1 of them up front); returns how many are running (mu_ held).
  unsigned grow(unsigned want) {
    while (started_ < want && started_ + 1 < kMaxCopyThreads) {
      try {
        std::thread([this] { run(); }).detach();
        started_++;
      } catch (...) {  // no thread available: split over the ones running
        break;
      }
    }
    return std::min(started_, want);
  }
  void run() {
    std::unique_lock<std::mutex> l(mu_);
    for (;;) {
      work_.wait(l, [&] { return !jobs_.empty(); });
      Job &j = *jobs_.front();
      const unsigned p = claim(j);
      l.unlock();
      piece(j, p);
      l.lock();
      // the caller returns (and its Job goes out of scope) only after seeing left == 0 under
      // mu_, so j stays valid up to here
      if (--j.left == 0) j.done.notify_one();
    }
  }
  unsigned cap_ = 1, started_ = 0;  // started_: guarded by mu_
  std::mutex mu_;
  std::condition_variable work_;
  std::deque<Job *> jobs_;  // posted jobs with unclaimed pieces, oldest first
  std::atomic<unsigned> inflight_{0}, max_inflight_{0};
};

}  // namespace nttmul
