// queue_host.cpp — TEST ONLY: the product's batching queue (at2-node_amd/csrc/at2v_queue.h) driven on
// the CPU with the oracle as its verify backend, to check flush policy, ticket order and verdict mapping
// without a GPU. The shipped queue is instantiated with the HIP backend in at2v_host.hip.
// usage: queue_host <scenario>   scenario in {order, size, deadline, flush, eager, eager_order, drain, startfail, failed}; exit 0 = pass
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "at2v_queue.h"
#include "../../oracle/ed25519_oracle.h"

using namespace at2v;

struct OracleBackend {
  std::atomic<int> launches{0};
  int fail_alloc_at = -1;   // >= 0: the alloc() call with this index fails after taking one buffer
  int fail_launch_at = -1;  // >= 0: the launch() call with this index reports a device error
  int allocs = 0, releases = 0, held = 0;  // buffers taken and given back (leak check)
  int alloc(QueueSlot& s) {
    if (allocs++ == fail_alloc_at) {
      s.pk = (uint8_t*)malloc(s.cap_records * 32);  // partly allocated slot
      held += s.pk != nullptr;
      return -4;
    }
    s.pk = (uint8_t*)malloc(s.cap_records * 32);
    s.sig = (uint8_t*)malloc(s.cap_records * 64);
    s.msg = (uint8_t*)malloc(s.cap_msg);
    s.off = (uint32_t*)malloc((s.cap_records + 1) * 4);
    s.verdicts = (uint32_t*)malloc((s.cap_records + 31) / 32 * 4);
    held += 5;
    return (s.pk && s.sig && s.msg && s.off && s.verdicts) ? 0 : -4;
  }
  void release(QueueSlot& s) {
    ++releases;
    for (void* p : {(void*)s.pk, (void*)s.sig, (void*)s.msg, (void*)s.off, (void*)s.verdicts}) held -= p != nullptr;
    free(s.pk);
    free(s.sig);
    free(s.msg);
    free(s.off);
    free(s.verdicts);
  }
  int launch(QueueSlot& s) {  // asynchronous, like the HIP backend
    if (launches++ == fail_launch_at) return -3;
    s.backend = new std::thread([&s] {
      oracle_verify_batch(s.pk, s.sig, s.msg, s.off, s.n, ORACLE_POLICY_DALEK_V1, s.verdicts, 2);
    });
    return 0;
  }
  int wait(QueueSlot& s) {
    auto* t = static_cast<std::thread*>(s.backend);
    if (!t) return -3;
    t->join();
    delete t;
    s.backend = nullptr;
    return 0;
  }
};

#define REQUIRE(c)                                                  \
  do {                                                              \
    if (!(c)) {                                                     \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                     \
    }                                                               \
  } while (0)

struct Records {
  size_t n, L;
  std::vector<uint8_t> pk, sig, msg, cls;
  std::vector<uint32_t> off;
  std::vector<uint8_t> want;
  Records(size_t n_, size_t L_) : n(n_), L(L_), pk(n * 32), sig(n * 64), msg(n * L), cls(n), off(n + 1), want(n) {
    oracle_gen_adversarial(0x51, 0, n, L, pk.data(), sig.data(), msg.data(), cls.data(), 8);
    for (size_t i = 0; i <= n; ++i) off[i] = (uint32_t)(i * L);
    for (size_t i = 0; i < n; ++i)
      want[i] = (uint8_t)oracle_verify(&pk[32 * i], &sig[64 * i], &msg[L * i], L, ORACLE_POLICY_DALEK_V1);
  }
};

static long drain(BatchQueue<OracleBackend>& q, std::vector<uint8_t>& got, std::vector<uint64_t>& order, size_t want,
                  uint32_t timeout_us) {
  std::vector<uint64_t> t(1024);
  std::vector<uint8_t> v(1024);
  const uint64_t t0 = now_us();
  while (order.size() < want && now_us() - t0 < timeout_us) {
    const long k = q.poll(t.data(), v.data(), t.size(), 20000);
    for (long i = 0; i < k; ++i) {
      order.push_back(t[i]);
      if (t[i] < got.size()) got[t[i]] = v[i];
    }
  }
  return (long)order.size();
}

int scenario_order() {
  // 4 producers submit random-size runs; tickets map back to records; polled in ticket order
  Records r(6000, 77);
  OracleBackend be;
  QueueOpts o;
  o.max_batch = 500;
  o.max_delay_us = 2000;
  o.max_msg_bytes = 80;
  o.depth = 3;
  BatchQueue<OracleBackend> q(be, o);
  REQUIRE(q.start() == 0);
  std::vector<uint64_t> ticket_of(r.n, UINT64_MAX);
  std::atomic<size_t> next{0};
  std::vector<std::thread> th;
  for (int p = 0; p < 4; ++p)
    th.emplace_back([&, p] {
      std::mt19937 rng(p);
      while (true) {
        const size_t len = 1 + rng() % 97;
        const size_t a = next.fetch_add(len);
        if (a >= r.n) break;
        const size_t m = std::min(len, r.n - a);
        std::vector<uint32_t> off(m + 1);
        for (size_t i = 0; i <= m; ++i) off[i] = (uint32_t)(i * r.L);
        uint64_t first;
        if (q.submit(&r.pk[32 * a], &r.sig[64 * a], &r.msg[r.L * a], off.data(), m, &first) != 0) abort();
        for (size_t i = 0; i < m; ++i) ticket_of[a + i] = first + i;
      }
    });
  for (auto& t : th) t.join();
  q.flush();
  std::vector<uint8_t> got(r.n, 0xee);
  std::vector<uint64_t> order;
  const long nd = drain(q, got, order, r.n, 60000000);
  if (nd != (long)r.n) {
    const QueueStats s = q.stats();
    fprintf(stderr, "drained %ld of %zu; submitted %llu completed %llu batches %llu\n", nd, r.n,
            (unsigned long long)s.submitted, (unsigned long long)s.completed, (unsigned long long)s.batches);
  }
  REQUIRE(nd == (long)r.n);
  for (size_t i = 0; i < order.size(); ++i) REQUIRE(order[i] == i);  // ticket order
  size_t bad = 0, valid = 0;
  for (size_t i = 0; i < r.n; ++i) {
    REQUIRE(ticket_of[i] != UINT64_MAX);
    bad += got[ticket_of[i]] != r.want[i];
    valid += r.want[i];
  }
  const QueueStats s = q.stats();
  printf("order n=%zu valid=%zu mismatches=%zu batches=%llu mean_batch=%.1f\n", r.n, valid, bad,
         (unsigned long long)s.batches, s.mean_batch);
  REQUIRE(bad == 0 && valid > 0 && valid < r.n);
  REQUIRE(s.completed == r.n && s.submitted == r.n);
  return 0;
}

int scenario_size() {
  // a full batch is sealed at max_batch records without waiting for the (long) deadline
  Records r(1024, 48);
  OracleBackend be;
  QueueOpts o;
  o.max_batch = 256;
  o.max_delay_us = 30000000;
  o.max_msg_bytes = 48;
  o.depth = 2;
  BatchQueue<OracleBackend> q(be, o);
  REQUIRE(q.start() == 0);
  const uint64_t t0 = now_us();
  REQUIRE(q.submit(r.pk.data(), r.sig.data(), r.msg.data(), r.off.data(), r.n, nullptr) == 0);
  std::vector<uint8_t> got(r.n, 0xee);
  std::vector<uint64_t> order;
  REQUIRE(drain(q, got, order, r.n, 20000000) == (long)r.n);
  const uint64_t dt = now_us() - t0;
  const QueueStats s = q.stats();
  printf("size batches=%llu mean=%.1f dt_us=%llu\n", (unsigned long long)s.batches, s.mean_batch,
         (unsigned long long)dt);
  REQUIRE(s.batches == 4 && s.mean_batch == 256.0);
  REQUIRE(dt < 20000000);
  for (size_t i = 0; i < r.n; ++i) REQUIRE(got[i] == r.want[i]);
  return 0;
}

int scenario_deadline() {
  // a partial batch is sealed once its oldest record is max_delay_us old
  Records r(10, 64);
  OracleBackend be;
  QueueOpts o;
  o.max_batch = 65536;
  o.max_delay_us = 3000;
  o.max_msg_bytes = 64;
  o.depth = 2;
  BatchQueue<OracleBackend> q(be, o);
  REQUIRE(q.start() == 0);
  const uint64_t t0 = now_us();
  REQUIRE(q.submit(r.pk.data(), r.sig.data(), r.msg.data(), r.off.data(), r.n, nullptr) == 0);
  std::vector<uint8_t> got(r.n, 0xee);
  std::vector<uint64_t> order;
  REQUIRE(drain(q, got, order, r.n, 5000000) == (long)r.n);
  const uint64_t dt = now_us() - t0;
  const QueueStats s = q.stats();
  printf("deadline dt_us=%llu batches=%llu p50_us=%.0f\n", (unsigned long long)dt, (unsigned long long)s.batches,
         s.p50_us);
  REQUIRE(s.batches == 1 && dt >= 3000 && dt < 2000000);
  for (size_t i = 0; i < r.n; ++i) REQUIRE(got[i] == r.want[i]);
  return 0;
}

int scenario_eager() {
  // eager (latency) mode: with nothing in flight a lone record is launched at once, not at the deadline; records
  // that arrive while a batch verifies form the next batch
  Records r(40, 48);
  OracleBackend be;
  QueueOpts o;
  o.max_batch = 4096;
  o.max_delay_us = 30000000;  // 30 s: only the eager rule can seal within the test
  o.max_msg_bytes = 48;
  o.depth = 3;
  o.eager = true;
  BatchQueue<OracleBackend> q(be, o);
  REQUIRE(q.start() == 0);
  std::vector<uint8_t> got(r.n, 0xee);
  std::vector<uint64_t> order;
  const uint64_t t0 = now_us();
  REQUIRE(q.submit(r.pk.data(), r.sig.data(), r.msg.data(), r.off.data(), 1, nullptr) == 0);
  REQUIRE(drain(q, got, order, 1, 5000000) == 1);
  const uint64_t dt1 = now_us() - t0;
  // a burst of single-record submits: fewer batches than records, every verdict in ticket order
  for (size_t i = 1; i < r.n; ++i) {
    std::vector<uint32_t> o1 = {0, (uint32_t)r.L};
    REQUIRE(q.submit(&r.pk[32 * i], &r.sig[64 * i], &r.msg[r.L * i], o1.data(), 1, nullptr) == 0);
  }
  REQUIRE(drain(q, got, order, r.n, 20000000) == (long)r.n);
  const QueueStats s = q.stats();
  printf("eager first_us=%llu batches=%llu mean_batch=%.2f\n", (unsigned long long)dt1, (unsigned long long)s.batches,
         s.mean_batch);
  REQUIRE(dt1 < 5000000);
  REQUIRE(s.batches >= 2 && s.batches < r.n);
  for (size_t i = 0; i < r.n; ++i) REQUIRE(got[i] == r.want[i] && order[i] == i);
  return 0;
}

int scenario_eager_order() {
  // eager mode with 4 producers: batches are launched by producers, the completer and the launcher thread alike;
  // tickets still map back to records and verdicts come back in ticket order
  Records r(3000, 61);
  OracleBackend be;
  QueueOpts o;
  o.max_batch = 256;
  o.max_delay_us = 30000000;
  o.max_msg_bytes = 64;
  o.depth = 3;
  o.eager = true;
  BatchQueue<OracleBackend> q(be, o);
  REQUIRE(q.start() == 0);
  std::vector<uint64_t> ticket_of(r.n, UINT64_MAX);
  std::atomic<size_t> next{0};
  std::vector<std::thread> th;
  for (int p = 0; p < 4; ++p)
    th.emplace_back([&, p] {
      std::mt19937 rng(100 + p);
      while (true) {
        const size_t len = 1 + rng() % 9;
        const size_t a = next.fetch_add(len);
        if (a >= r.n) break;
        const size_t m = std::min(len, r.n - a);
        std::vector<uint32_t> off(m + 1);
        for (size_t i = 0; i <= m; ++i) off[i] = (uint32_t)(i * r.L);
        uint64_t first;
        if (q.submit(&r.pk[32 * a], &r.sig[64 * a], &r.msg[r.L * a], off.data(), m, &first) != 0) abort();
        for (size_t i = 0; i < m; ++i) ticket_of[a + i] = first + i;
      }
    });
  for (auto& t : th) t.join();
  std::vector<uint8_t> got(r.n, 0xee);
  std::vector<uint64_t> order;
  REQUIRE(drain(q, got, order, r.n, 60000000) == (long)r.n);
  for (size_t i = 0; i < order.size(); ++i) REQUIRE(order[i] == i);
  size_t bad = 0;
  for (size_t i = 0; i < r.n; ++i) {
    REQUIRE(ticket_of[i] != UINT64_MAX);
    bad += got[ticket_of[i]] != r.want[i];
  }
  const QueueStats s = q.stats();
  printf("eager_order n=%zu mismatches=%zu batches=%llu mean_batch=%.1f\n", r.n, bad, (unsigned long long)s.batches,
         s.mean_batch);
  REQUIRE(bad == 0 && s.completed == r.n && s.batches > 1);
  return 0;
}

int scenario_flush() {
  Records r(5, 32);
  OracleBackend be;
  QueueOpts o;
  o.max_batch = 1024;
  o.max_delay_us = 60000000;
  o.max_msg_bytes = 32;
  o.depth = 2;
  BatchQueue<OracleBackend> q(be, o);
  REQUIRE(q.start() == 0);
  std::vector<uint64_t> t(8);
  std::vector<uint8_t> v(8);
  REQUIRE(q.submit(r.pk.data(), r.sig.data(), r.msg.data(), r.off.data(), r.n, nullptr) == 0);
  REQUIRE(q.poll(t.data(), v.data(), 8, 50000) == 0);  // nothing sealed yet
  q.flush();
  std::vector<uint8_t> got(r.n, 0xee);
  std::vector<uint64_t> order;
  REQUIRE(drain(q, got, order, r.n, 5000000) == (long)r.n);
  for (size_t i = 0; i < r.n; ++i) REQUIRE(got[i] == r.want[i]);
  // empty flush and oversized messages are harmless / rejected
  q.flush();
  std::vector<uint32_t> big = {0, (uint32_t)(1024 * 32 + 1)};
  std::vector<uint8_t> mbig(big[1]);
  REQUIRE(q.submit(r.pk.data(), r.sig.data(), mbig.data(), big.data(), 1, nullptr) != 0);
  printf("flush ok\n");
  return 0;
}

int scenario_drain() {
  // stop() (destructor) completes everything that was submitted
  Records r(700, 40);
  OracleBackend be;
  QueueOpts o;
  o.max_batch = 300;
  o.max_delay_us = 60000000;
  o.max_msg_bytes = 40;
  o.depth = 3;
  QueueStats s;
  {
    BatchQueue<OracleBackend> q(be, o);
    REQUIRE(q.start() == 0);
    REQUIRE(q.submit(r.pk.data(), r.sig.data(), r.msg.data(), r.off.data(), r.n, nullptr) == 0);
    q.stop();
    s = q.stats();
  }
  printf("drain completed=%llu batches=%llu\n", (unsigned long long)s.completed, (unsigned long long)s.batches);
  REQUIRE(s.completed == r.n && s.batches == 3 && be.launches == 3);
  return 0;
}

int scenario_startfail() {
  // a start() that fails on slot 2 must not leak slots 0, 1 or the partial slot 2
  OracleBackend be;
  be.fail_alloc_at = 2;
  QueueOpts o;
  o.max_batch = 64;
  o.depth = 4;
  {
    BatchQueue<OracleBackend> q(be, o);
    REQUIRE(q.start() != 0);
  }  // destructor -> stop()
  printf("startfail allocs=%d releases=%d held=%d\n", be.allocs, be.releases, be.held);
  REQUIRE(be.allocs == 3 && be.held == 0);
  return 0;
}

int scenario_failed() {
  // a batch whose launch fails reports 0xff for each of its records (never 1), the others verify normally
  Records r(300, 48);
  OracleBackend be;
  be.fail_launch_at = 1;
  QueueOpts o;
  o.max_batch = 100;
  o.max_delay_us = 60000000;
  o.max_msg_bytes = 48;
  o.depth = 2;
  BatchQueue<OracleBackend> q(be, o);
  REQUIRE(q.start() == 0);
  REQUIRE(q.submit(r.pk.data(), r.sig.data(), r.msg.data(), r.off.data(), r.n, nullptr) == 0);
  std::vector<uint8_t> got(r.n, 0xee);
  std::vector<uint64_t> order;
  REQUIRE(drain(q, got, order, r.n, 20000000) == (long)r.n);
  for (size_t i = 0; i < r.n; ++i) REQUIRE(i / 100 == 1 ? got[i] == 0xff : got[i] == r.want[i]);
  const QueueStats s = q.stats();
  printf("failed batches=%llu failed_batches=%llu\n", (unsigned long long)s.batches,
         (unsigned long long)s.failed_batches);
  REQUIRE(s.batches == 3 && s.failed_batches == 1);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const char* s = argv[1];
  if (!strcmp(s, "order")) return scenario_order();
  if (!strcmp(s, "size")) return scenario_size();
  if (!strcmp(s, "deadline")) return scenario_deadline();
  if (!strcmp(s, "flush")) return scenario_flush();
  if (!strcmp(s, "eager")) return scenario_eager();
  if (!strcmp(s, "eager_order")) return scenario_eager_order();
  if (!strcmp(s, "drain")) return scenario_drain();
  if (!strcmp(s, "startfail")) return scenario_startfail();
  if (!strcmp(s, "failed")) return scenario_failed();
  return 2;
}
