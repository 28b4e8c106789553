// ThreadSanitizer driver of csrc/copy_pool.hpp (the host-buffer path's split staging memcpy,
// tests/test_sanitizers.py): several caller threads, as several contexts' host calls would, copy
// blocks of varied sizes with varied thread counts through the one process-wide pool at once, and
// every destination is checked byte for byte.  Any data race or lost wake-up fails the run (TSan
// report, or the 60 s alarm of a hang).  The callers start together, and the run reports the most
// split copies the pool had in flight at once: with argv[3] = k it fails unless some k of them
// overlapped (the pool no longer runs one split copy at a time, verdict r5 item 3).
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <thread>
#include <vector>

#include "copy_pool.hpp"

int main(int argc, char **argv) {
  alarm(60);
  const int callers = argc > 1 ? atoi(argv[1]) : 4;
  const int rounds = argc > 2 ? atoi(argv[2]) : 40;
  const unsigned need_overlap = argc > 3 ? (unsigned)atoi(argv[3]) : 0;
  std::atomic<int> bad{0}, ready{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < callers; t++) {
    ts.emplace_back([t, rounds, callers, &bad, &ready] {
      ready++;
      while (ready.load() < callers) std::this_thread::yield();  // start together
      unsigned seed = 0x9E3779B9u * (t + 1);
      auto rnd = [&seed] { return seed = seed * 1664525u + 1013904223u; };
      for (int r = 0; r < rounds; r++) {
        // below one part (plain memcpy), a few parts, sizes that are not a multiple of the 4 KiB
        // step rounding, and 3 MiB + 2 (advisor r5: bytes / parts a multiple of 4 KiB with a
        // remainder, which a floor split left uncopied)
        const size_t sizes[] = {4096, (size_t)3 << 20, ((size_t)5 << 20) + 12345, (size_t)9 << 20,
                                ((size_t)3 << 20) + 2};
        const size_t bytes = sizes[rnd() % 5];
        const unsigned threads = 1 + rnd() % 12;
        std::vector<unsigned char> src(bytes), dst(bytes, 0xEE);
        for (size_t i = 0; i < bytes; i++) src[i] = (unsigned char)(i * 131 + r * 7 + t);
        nttmul::CopyPool::get().copy(dst.data(), src.data(), bytes, threads);
        if (memcmp(dst.data(), src.data(), bytes) != 0) bad++;
      }
    });
  }
  for (auto &th : ts) th.join();
  if (bad) {
    printf("copy pool: %d mismatching copies\n", bad.load());
    return 1;
  }
  const unsigned overlap = nttmul::CopyPool::get().max_concurrent_splits();
  printf("max split copies in flight at once: %u (workers %u)\n", overlap,
         nttmul::CopyPool::get().workers());
  if (overlap < need_overlap) {
    printf("copy pool: split copies never overlapped (%u < %u)\n", overlap, need_overlap);
    return 1;
  }
  printf("copy pool tsan run ok (%d callers x %d copies)\n", callers, rounds);
  return 0;
}
