// Per-step agreements between the ranks of ONE node through host shared
// memory (the reference's two whole-complex decisions per hyperplane step:
// "does anything split" subpoly.py:110 and the failover override
// subpoly_debug.py:43-49, plus the OR of the ranks' next-active plane masks).
// A handful of int64 words per rank per step: a collective library call
// (RCCL all_gather + host copies, ~tens of microseconds) is mostly latency;
// here every rank writes its words into its slot, arrives on one atomic
// counter and spins until all have arrived (a few microseconds).
//
// Layout: a 64-B header holding the arrival counter, then two banks of
// world x SHM_WORDS int64 slots.  Call g (1, 2, ...) uses bank (g - 1) & 1: a rank can only
// rewrite a bank at call g + 2, after every rank arrived at call g + 1, i.e.
// after every rank has finished reading call g's bank -- one barrier per call.
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>

#include "../../include/tropical_hip.h"
#include "common.h"

namespace {
constexpr int SHM_WORDS = 16;  // (the curve branch: 8 convergence words + the failure word)
struct Hdr {
  std::atomic<uint64_t> arrive;
  char pad[56];
};
}  // namespace

struct tnp_shm {
  int fd = -1;
  void* base = nullptr;
  size_t bytes = 0;
  int rank = 0, world = 1;
  uint64_t gen = 0;
};

static size_t shm_bytes(int world) { return sizeof(Hdr) + 2ull * world * SHM_WORDS * sizeof(int64_t); }

extern "C" int tnp_shm_open(const char* name, int rank, int world, int create, tnp_shm** out) {
  if (world < 1 || rank < 0 || rank >= world || !name || name[0] != '/') {
    tnp_set_error("tnp_shm_open: bad arguments (rank %d, world %d, name %s)", rank, world, name ? name : "-");
    return -1;
  }
  const size_t bytes = shm_bytes(world);
  int fd;
  if (create) {
    shm_unlink(name);  // a stale segment of a killed run
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd >= 0 && ftruncate(fd, (off_t)bytes) != 0) {
      close(fd);
      fd = -1;
    }
  } else {
    fd = shm_open(name, O_RDWR, 0600);
  }
  if (fd < 0) {
    tnp_set_error("tnp_shm_open: shm_open(%s) failed", name);
    return -1;
  }
  void* base = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (base == MAP_FAILED) {
    close(fd);
    tnp_set_error("tnp_shm_open: mmap failed");
    return -1;
  }
  if (create) {
    memset(base, 0, bytes);
    new (base) Hdr();
  }
  tnp_shm* s = new tnp_shm();
  s->fd = fd;
  s->base = base;
  s->bytes = bytes;
  s->rank = rank;
  s->world = world;
  *out = s;
  return 0;
}

extern "C" int tnp_shm_unlink(const char* name) {
  return shm_unlink(name) == 0 ? 0 : -1;
}

extern "C" void tnp_shm_close(tnp_shm* s) {
  if (!s) return;
  if (s->base) munmap(s->base, s->bytes);
  if (s->fd >= 0) close(s->fd);
  delete s;
}

extern "C" int tnp_shm_allreduce(tnp_shm* s, const int64_t* in, int n, int op, int64_t* out) {
  if (n < 1 || n > SHM_WORDS || (op != TNP_SHM_MAX && op != TNP_SHM_OR && op != TNP_SHM_SUM && op != TNP_SHM_AND)) {
    tnp_set_error("tnp_shm_allreduce: %d words (max %d), op %d", n, SHM_WORDS, op);
    return -1;
  }
  Hdr* h = static_cast<Hdr*>(s->base);
  int64_t* bank = reinterpret_cast<int64_t*>(static_cast<char*>(s->base) + sizeof(Hdr)) +
                  (size_t)(s->gen & 1) * s->world * SHM_WORDS;
  const uint64_t g = ++s->gen;
  memcpy(bank + (size_t)s->rank * SHM_WORDS, in, n * sizeof(int64_t));
  h->arrive.fetch_add(1, std::memory_order_acq_rel);
  const uint64_t want = g * (uint64_t)s->world;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spin = 0; h->arrive.load(std::memory_order_acquire) < want; ++spin) {
    if (spin > 4096) sched_yield();  // oversubscribed cores: let the others arrive
    if ((spin & 0xFFFF) == 0xFFFF &&
        std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) {
      tnp_set_error("tnp_shm_allreduce: ranks did not arrive within 120 s (call %llu)", (unsigned long long)g);
      return -1;
    }
  }
  for (int k = 0; k < n; ++k) {
    int64_t v = bank[k];
    for (int r = 1; r < s->world; ++r) {
      const int64_t w = bank[(size_t)r * SHM_WORDS + k];
      v = op == TNP_SHM_MAX ? (w > v ? w : v) : op == TNP_SHM_OR ? (v | w) : op == TNP_SHM_AND ? (v & w) : v + w;
    }
    out[k] = v;
  }
  return 0;
}
