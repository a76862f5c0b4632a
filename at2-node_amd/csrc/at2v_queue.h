// at2v_queue.h — transaction ingest/batching queue in front of the batch verifier.
//
// In the reference, every payload that arrives through the sieve/contagion broadcast
// (/root/reference/src/bin/server/rpc.rs:275-284) is verified on its own by drop::crypto::sign on one of
// num_cpus::get() workers (rpc.rs:125), and the verified payloads come back in batches through
// deliver() (rpc.rs:156-173). This queue is the MI355X-side replacement of that per-payload step:
//   * producers submit records (A, R||S, M) and get monotonically increasing tickets;
//   * a launcher thread seals the filling batch when it holds `max_batch` records, when its oldest
//     record is `max_delay_us` old, or on flush(), and starts an asynchronous verify of it; in eager
//     mode it also seals as soon as no batch is in flight (latency mode: a lone record is launched at
//     once, and records arriving during a verify form the next batch, so batch size follows the load);
//   * a completer thread waits for batches in launch order and publishes (ticket, verdict) in ticket
//     order, so verdicts map back to payloads without any per-record bookkeeping by the caller;
//   * `depth` batch slots: one filling while up to depth-1 are in flight (copy/compute overlap).
// Header-only over a Backend (launch/wait on a slot) so the same queue logic is exercised on the CPU by
// tests/host/queue_host.cpp; the product instantiates it with the HIP backend (at2v_host.hip).
#pragma once
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

namespace at2v {

inline uint64_t now_us() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct QueueOpts {
  size_t max_batch = 65536;    // records per batch (slot capacity)
  uint32_t max_delay_us = 1000;
  size_t max_msg_bytes = 256;  // average message bytes budgeted per record (slot msg capacity = max_batch x this)
  int depth = 3;               // slots: 1 filling + up to depth-1 in flight
  bool eager = false;          // also seal whenever the device is idle (no batch in flight)
  bool launch_here = true;     // eager: the producer / completer that finds the device idle launches the batch itself
};

struct QueueSlot {
  // host buffers (pinned in the HIP backend), ABI layout of at2v_verify_batch
  uint8_t* pk = nullptr;
  uint8_t* sig = nullptr;
  uint8_t* msg = nullptr;
  uint32_t* off = nullptr;
  uint32_t* verdicts = nullptr;
  size_t cap_records = 0, cap_msg = 0;
  size_t n = 0, msg_used = 0;
  uint64_t first_ticket = 0;
  uint64_t t_first = 0;
  std::vector<std::pair<uint32_t, uint64_t>> t_runs;  // (records, submit time) per submit call
  int status = 0;
  void* backend = nullptr;
};

struct QueueStats {
  uint64_t submitted = 0, completed = 0, batches = 0, failed_batches = 0;
  double mean_batch = 0, p50_us = 0, p99_us = 0, max_us = 0;
};

template <class Backend>
class BatchQueue {
 public:
  BatchQueue(Backend& be, const QueueOpts& o) : be_(be), o_(o) {}
  ~BatchQueue() { stop(); }

  int start() {
    if (o_.depth < 2 || o_.max_batch == 0) return -1;
    slots_.resize(o_.depth);
    for (auto& s : slots_) {
      s.cap_records = o_.max_batch;
      s.cap_msg = std::max<size_t>(o_.max_batch * o_.max_msg_bytes, 64);
      const int e = be_.alloc(s);
      if (e) return e;
      free_.push_back(&s);
    }
    running_ = true;
    launcher_ = std::thread([this] { launcher_loop(); });
    completer_ = std::thread([this] { completer_loop(); });
    return 0;
  }

  // Seals what is pending, waits until every launched batch has completed, joins the threads, frees the
  // slots. Also frees what a start() that failed part-way had allocated (no threads were started then).
  void stop() {
    {
      std::unique_lock<std::mutex> lk(m_);
      if (!running_) {
        lk.unlock();
        release_slots();
        return;
      }
      flush_req_ = true;
      cv_launch_.notify_all();
      cv_idle_.wait(lk, [&] { return (!fill_ || fill_->n == 0) && ready_.empty() && !launching_ && inflight_.empty(); });
      running_ = false;
    }
    cv_launch_.notify_all();
    cv_complete_.notify_all();
    launcher_.join();
    completer_.join();
    release_slots();
  }

  // Append n records (ABI layout; msg_off has n+1 entries, message i = msg[off[i]..off[i+1])).
  int submit(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint32_t* off, size_t n,
             uint64_t* first_ticket) {
    // one call's records get consecutive tickets: producers are serialised for the whole call (a call
    // may block for a free slot, and nobody else may take tickets meanwhile)
    std::lock_guard<std::mutex> producer(submit_m_);
    std::unique_lock<std::mutex> lk(m_);
    if (!running_) return -1;
    for (size_t i = 0; i < n; ++i)  // validate the whole call before taking any record
      if (off[i + 1] < off[i] || off[i + 1] - off[i] > slots_[0].cap_msg) return -1;
    if (first_ticket) *first_ticket = next_ticket_;
    const uint64_t t = now_us();  // one submit time for the whole call
    size_t i = 0;
    while (i < n) {
      if (fill_ && (fill_->n == fill_->cap_records || fill_->msg_used + (off[i + 1] - off[i]) > fill_->cap_msg))
        seal_locked();
      if (!fill_) {
        cv_free_.wait(lk, [&] { return fill_ || !free_.empty() || !running_; });
        if (!running_) return -1;
      }
      if (!fill_) {
        fill_ = free_.front();
        free_.pop_front();
        fill_->n = 0;
        fill_->msg_used = 0;
        fill_->first_ticket = next_ticket_;
        fill_->t_runs.clear();
        fill_->off[0] = 0;
      }
      QueueSlot& s = *fill_;
      if (s.n == 0) {
        s.t_first = t;
        cv_launch_.notify_all();  // arm the deadline
      }
      // bulk-copy the longest run of records that fits the slot (records and message bytes)
      size_t m = std::min(n - i, s.cap_records - s.n);
      const size_t room = s.cap_msg - s.msg_used;
      if (off[i + m] - off[i] > room) {  // offsets are non-decreasing: binary search the message-byte limit
        size_t lo = 1, hi = m;             // off[i+1]-off[i] <= room holds (checked above)
        while (lo < hi) {
          const size_t mid = (lo + hi + 1) / 2;
          if (off[i + mid] - off[i] <= room) lo = mid; else hi = mid - 1;
        }
        m = lo;
      }
      const uint32_t mb = off[i + m] - off[i];
      std::memcpy(s.pk + 32 * s.n, pk + 32 * i, 32 * m);
      std::memcpy(s.sig + 64 * s.n, sig + 64 * i, 64 * m);
      if (mb) std::memcpy(s.msg + s.msg_used, msg + off[i], mb);
      const uint32_t base = (uint32_t)s.msg_used - off[i];
      for (size_t k = 1; k <= m; ++k) s.off[s.n + k] = off[i + k] + base;
      s.msg_used += mb;
      s.n += m;
      s.t_runs.emplace_back((uint32_t)m, t);
      next_ticket_ += m;
      stats_.submitted += m;
      i += m;
      if (s.n == s.cap_records) seal_locked();
    }
    // latency mode with the device idle: this thread seals and launches the batch itself instead of waking the
    // launcher thread (one thread hand-off less per lone batch); if a launch is under way the launcher takes it
    if (o_.eager && o_.launch_here && fill_ && fill_->n && ready_.empty() && inflight_.empty() && !launching_) {
      seal_locked();
      launch_here_locked(lk);
    }
    return 0;
  }

  // Seal the filling batch now (non-blocking).
  void flush() {
    std::lock_guard<std::mutex> lk(m_);
    if (fill_ && fill_->n) seal_locked();
  }

  // Up to `max` completed (ticket, verdict) pairs in ticket order; waits up to timeout_us for the first.
  long poll(uint64_t* tickets, uint8_t* verdicts, size_t max, uint32_t timeout_us) {
    std::unique_lock<std::mutex> lk(m_);
    if (done_.empty() && timeout_us)
      cv_done_.wait_for(lk, std::chrono::microseconds(timeout_us), [&] { return !done_.empty(); });
    size_t k = 0;
    while (k < max && !done_.empty()) {
      Done& d = done_.front();
      while (k < max && d.used < d.n) {
        const size_t i = d.used++;
        tickets[k] = d.first + i;
        verdicts[k] = d.failed ? 0xff : (uint8_t)((d.words[i >> 5] >> (i & 31)) & 1u);
        ++k;
      }
      if (d.used == d.n) done_.pop_front();
    }
    return (long)k;
  }

  QueueStats stats() {
    std::lock_guard<std::mutex> lk(m_);
    QueueStats s = stats_;
    s.mean_batch = s.batches ? (double)s.completed / (double)s.batches : 0.0;
    if (!lat_.empty()) {
      std::vector<uint32_t> v(lat_);
      auto pct = [&](double q) {
        const size_t i = std::min(v.size() - 1, (size_t)(q * (double)(v.size() - 1) + 0.5));
        std::nth_element(v.begin(), v.begin() + i, v.end());
        return (double)v[i];
      };
      s.p50_us = pct(0.50);
      s.p99_us = pct(0.99);
      s.max_us = (double)*std::max_element(v.begin(), v.end());
    }
    return s;
  }

  void reset_latency() {
    std::lock_guard<std::mutex> lk(m_);
    lat_.clear();
  }

 private:
  struct Done {
    uint64_t first;
    size_t n, used;
    bool failed;
    std::vector<uint32_t> words;
  };

  // every slot that start() touched, including a partly allocated one (release() skips null buffers)
  void release_slots() {
    for (auto& s : slots_) be_.release(s);
    slots_.clear();
    free_.clear();
  }

  void seal_locked() {
    ready_.push_back(fill_);
    fill_ = nullptr;
    cv_launch_.notify_all();
  }

  // Launch the oldest sealed batch. Caller holds m_ (lk) and launch_m_; m_ is released around the backend call. Every
  // launch runs under launch_m_ and pops/pushes under m_, so launch order = seal order = ticket order whichever
  // thread launches.
  void launch_one_locked(std::unique_lock<std::mutex>& lk) {
    QueueSlot* s = ready_.front();
    ready_.pop_front();
    ++launching_;
    lk.unlock();
    s->status = be_.launch(*s);
    lk.lock();
    --launching_;
    inflight_.push_back(s);
    cv_complete_.notify_all();
  }

  // From a producer or the completer (holding m_): launch what is sealed if no other thread is launching; never
  // blocks on launch_m_ while holding m_ (the launcher thread takes launch_m_ before m_).
  void launch_here_locked(std::unique_lock<std::mutex>& lk) {
    if (ready_.empty() || !launch_m_.try_lock()) return;
    std::lock_guard<std::mutex> g(launch_m_, std::adopt_lock);
    while (!ready_.empty()) launch_one_locked(lk);
  }

  void launcher_loop() {
    std::unique_lock<std::mutex> lk(m_);
    while (true) {
      if (fill_ && fill_->n) {
        const bool idle = inflight_.empty() && ready_.empty() && !launching_;
        if (flush_req_ || now_us() >= fill_->t_first + o_.max_delay_us || (o_.eager && idle)) seal_locked();
      }
      if (flush_req_ && (!fill_ || fill_->n == 0)) flush_req_ = false;
      if (!ready_.empty()) {
        lk.unlock();
        std::lock_guard<std::mutex> g(launch_m_);  // (launch_m_ before m_: see launch_here_locked)
        lk.lock();
        if (!ready_.empty()) launch_one_locked(lk);
        continue;
      }
      if (!running_) break;
      if (fill_ && fill_->n) {
        const auto dl = std::chrono::steady_clock::time_point(std::chrono::microseconds(fill_->t_first + o_.max_delay_us));
        cv_launch_.wait_until(lk, dl);
      } else {
        cv_launch_.wait(lk);
      }
    }
  }

  void completer_loop() {
    std::unique_lock<std::mutex> lk(m_);
    while (true) {
      cv_complete_.wait(lk, [&] { return !inflight_.empty() || !running_; });
      if (inflight_.empty()) {
        if (!running_) break;
        continue;
      }
      QueueSlot* s = inflight_.front();
      lk.unlock();
      int st = s->status;
      if (st == 0) st = be_.wait(*s);
      const uint64_t t = now_us();
      lk.lock();
      inflight_.pop_front();
      Done d{s->first_ticket, s->n, 0, st != 0, {}};
      d.words.assign(s->verdicts, s->verdicts + (s->n + 31) / 32);
      done_.push_back(std::move(d));
      for (const auto& r : s->t_runs) {
        const uint32_t d = (uint32_t)std::min<uint64_t>(t - r.second, UINT32_MAX);
        const size_t k = std::min<size_t>(r.first, kMaxLatencySamples - std::min(kMaxLatencySamples, lat_.size()));
        lat_.insert(lat_.end(), k, d);
      }
      stats_.completed += s->n;
      ++stats_.batches;
      if (st) ++stats_.failed_batches;
      s->n = 0;
      free_.push_back(s);
      cv_free_.notify_all();
      cv_done_.notify_all();
      if (o_.eager && o_.launch_here && fill_ && fill_->n && ready_.empty() && inflight_.empty() && !launching_) {
        seal_locked();  // the device went idle: seal what is filling and launch it from here
        launch_here_locked(lk);
      } else if (o_.eager) {
        cv_launch_.notify_all();
      }
      if ((!fill_ || fill_->n == 0) && ready_.empty() && !launching_ && inflight_.empty()) cv_idle_.notify_all();
    }
  }

  static constexpr size_t kMaxLatencySamples = 1u << 22;
  Backend& be_;
  QueueOpts o_;
  std::vector<QueueSlot> slots_;
  std::deque<QueueSlot*> free_, ready_, inflight_;
  QueueSlot* fill_ = nullptr;
  std::deque<Done> done_;
  std::vector<uint32_t> lat_;
  QueueStats stats_;
  uint64_t next_ticket_ = 0;
  int launching_ = 0;
  bool running_ = false, flush_req_ = false;
  std::mutex m_, submit_m_, launch_m_;
  std::condition_variable cv_launch_, cv_complete_, cv_free_, cv_done_, cv_idle_;
  std::thread launcher_, completer_;
};

}  // namespace at2v
