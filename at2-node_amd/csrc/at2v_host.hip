// at2v_host.hip — C ABI of the host-side pieces around the verify kernel (include/at2v.h):
//   * at2v_queue_*   ingest/batching queue (at2v_queue.h) over a HIP backend: pinned host slots, one stream for
//                    H2D copies, two alternating verify streams and one for D2H copies, so batch k+1 uploads while
//                    batch k verifies, and batch k+1's kernel fills the CUs batch k's kernel leaves at its end (the
//                    context's scratch sets, at2v_api.hip);
//   * at2v_pack_*    SendAssetRequest -> verify records (at2v_pack.h);
//   * at2v_ledger_*  accounts / recent transactions / apply loop (at2v_ledger.h).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <new>

#include "../../include/at2v.h"
#include "at2v_env.h"
#include "at2v_ledger.h"
#include "at2v_pack.h"
#include "at2v_queue.h"

namespace {

// A slot's host buffers are ONE pinned allocation and its device buffers ONE device allocation with the same layout
// [pk cap x 32 | sig cap x 64 | off (cap + 1) x 4 | msg cap_msg], so a batch whose used span (the record arrays up to
// the capacity, plus the used message bytes) is small goes up in a single copy instead of four (kSingleCopyMax).
struct DevSlot {
  uint8_t* dev = nullptr;  // device allocation
  uint8_t* host = nullptr; // pinned host allocation (slot.pk points at its start)
  size_t msg_at = 0;       // byte offset of msg in both allocations
  void *pk = nullptr, *sig = nullptr, *msg = nullptr, *off = nullptr, *ver = nullptr;
  hipEvent_t uploaded = nullptr, verified = nullptr, done = nullptr;
  hipStream_t stream = nullptr;  // the compute stream of the slot's last launch
  bool cpu_done = false;         // the slot's batch was verified on the CPU backend (AT2V_QUEUE_CPU[_FALLBACK])
};
constexpr size_t kSingleCopyMax = 2u << 20;

// Sets the queue's device for a scope and restores the caller's current device on every return path: with launches from
// the producer's thread (at2v_queue_submit in latency mode) a user thread must not find its HIP device switched
// (ADVICE r4).
struct DeviceScope {
  int prev = -1;
  hipError_t err;
  explicit DeviceScope(int device) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    err = prev == device ? hipSuccess : hipSetDevice(device);
  }
  ~DeviceScope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

struct HipBackend {
  at2v_ctx* ctx = nullptr;
  int device = 0;
  // AT2V_QUEUE_CPU: ctx is a CPU context (num_gpus = 0) and every batch is verified on it, synchronously in launch().
  // AT2V_QUEUE_CPU_FALLBACK: cpu_ctx is a CPU context beside the GPU one; a batch whose launch or completion fails on the
  // device is verified there from the slot's host records (the verdict words are the slot's pinned host words).
  bool cpu_only = false;
  at2v_ctx* cpu_ctx = nullptr;
  std::atomic<uint64_t> fallbacks{0};
  // three streams of the queue + the context's own (which runs the sender-cache builds): four, one hardware queue each
  // (GPU_MAX_HW_QUEUES = 4), so no verify or copy of the latency path waits behind a comb build in a shared queue
  hipStream_t h2d = nullptr, comp[2] = {nullptr, nullptr};
  unsigned launches = 0;
  // the kernel writes the verdict words straight into the slot's pinned host words (no device-to-host copy after the
  // kernel: one dependent copy less on the latency path); AT2V_QUEUE_DIRECT=0 restores the copy (A/B)
  bool direct = true;
  // AT2V_QUEUE_SPIN_US > 0: the completer polls the batch's event for up to that long before the blocking wait. Off:
  // on MI355X the blocking wait already returns as fast (config 5 queue p50 within 2 us either way, profiles/r04v).
  uint32_t spin_us = 0;
  // Batches of at most zerocopy_max records are not uploaded: the kernel reads the slot's pinned host buffers directly
  // (one host-to-device copy and its cross-stream wait less on the latency path; config 5 queue p50 123-130 -> 109-117
  // us, p99 242-285 -> 154-187 us, profiles/r04w). AT2V_QUEUE_ZEROCOPY overrides (0 = always upload).
  uint32_t zerocopy_max = 1024;
  // Compute streams the queue alternates over: 2 in throughput mode (batch k+1's kernel fills the CUs batch k's leaves),
  // 1 in latency mode (AT2V_QUEUE_EAGER: batches are small and rarely overlap). AT2V_QUEUE_STREAMS overrides (1 or 2),
  // AT2V_QUEUE_PRIORITY = 1 gives them the device's greatest stream priority (A/B). The host-to-device stream is
  // created on the first batch that needs an upload (above zerocopy_max records). A latency-mode node so maps two
  // hardware queues (its stream and the context's), not four: with another process holding an RCCL communicator and six
  // streams on the same GPU, config-5 p99 was 0.70-0.97 ms per node with four and 0.56 ms with two, as without that
  // process (0.54-0.56 ms); priority changed nothing (profiles/r05f).
  int ncomp = 2;
  bool prio = false;

  int init(const at2v_queue_opts& o) {
    at2v_opts co{o.device, 1, o.policy, 0, 0, 0, o.cpu_threads, 0};
    if (o.flags & AT2V_QUEUE_CPU) {
      cpu_only = true;
      co.num_gpus = 0;
      return at2v_create(&co, &ctx);
    }
    if (o.flags & AT2V_QUEUE_SENDER_COMB) {
      co.sender_cache = o.sender_cache ? o.sender_cache : 1024u;
      co.sender_comb = 1;
    }
    int rc = at2v_create(&co, &ctx);
    if (rc) return rc;
    if (o.flags & AT2V_QUEUE_CPU_FALLBACK) {
      at2v_opts cc{0, 0, o.policy, 0, 0, 0, o.cpu_threads, 0};
      rc = at2v_create(&cc, &cpu_ctx);
      if (rc) return rc;
    }
    device = o.device;
    if (const char* v = at2v::test_env("AT2V_QUEUE_DIRECT")) direct = std::atoi(v) != 0;
    if (const char* v = at2v::test_env("AT2V_QUEUE_ZEROCOPY")) zerocopy_max = (uint32_t)std::strtoul(v, nullptr, 10);
    if (const char* v = at2v::test_env("AT2V_QUEUE_SPIN_US")) spin_us = (uint32_t)std::strtoul(v, nullptr, 10);
    if (o.flags & AT2V_QUEUE_EAGER) ncomp = 1;
    if (const char* v = at2v::test_env("AT2V_QUEUE_STREAMS")) ncomp = std::atoi(v) == 1 ? 1 : 2;
    if (const char* v = at2v::test_env("AT2V_QUEUE_PRIORITY")) prio = std::atoi(v) != 0;
    const DeviceScope scope(device);
    if (scope.err != hipSuccess) return AT2V_E_HIP;
    int least = 0, greatest = 0;
    if (prio && hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) prio = false;
    for (int k = 0; k < ncomp; ++k) {
      const hipError_t e = prio ? hipStreamCreateWithPriority(&comp[k], hipStreamNonBlocking, greatest)
                                : hipStreamCreateWithFlags(&comp[k], hipStreamNonBlocking);
      if (e != hipSuccess) return AT2V_E_HIP;
    }
    return AT2V_OK;
  }
  void fini() {
    at2v_destroy(cpu_ctx);
    cpu_ctx = nullptr;
    if (cpu_only) {
      at2v_destroy(ctx);
      ctx = nullptr;
      return;
    }
    const DeviceScope scope(device);
    if (scope.err == hipSuccess) {
      for (hipStream_t* s : {&h2d, &comp[0], &comp[1]})
        if (*s) {
          (void)hipStreamSynchronize(*s);
          (void)hipStreamDestroy(*s);
          *s = nullptr;
        }
    }
    at2v_destroy(ctx);
    ctx = nullptr;
  }

  int alloc(at2v::QueueSlot& s) {
    DevSlot* d = new (std::nothrow) DevSlot;
    if (!d) return AT2V_E_OOM;
    s.backend = d;
    const size_t words = (s.cap_records + 31) / 32;
    const size_t cap = s.cap_records;
    d->msg_at = (cap * 100 + 4 + 15) / 16 * 16;  // pk, sig, off, then msg 16-byte aligned
    const size_t bytes = d->msg_at + s.cap_msg + 16;
    if (cpu_only) {  // host memory only
      d->host = static_cast<uint8_t*>(std::malloc(bytes));
      s.verdicts = static_cast<uint32_t*>(std::malloc(words * 4));
      if (!d->host || !s.verdicts) return AT2V_E_OOM;
      s.pk = d->host;
      s.sig = d->host + cap * 32;
      s.off = reinterpret_cast<uint32_t*>(d->host + cap * 96);
      s.msg = d->host + d->msg_at;
      return AT2V_OK;
    }
    const DeviceScope scope(device);
    if (scope.err != hipSuccess) return AT2V_E_HIP;
    bool ok = hipHostMalloc((void**)&d->host, bytes, hipHostMallocDefault) == hipSuccess &&
              hipHostMalloc((void**)&s.verdicts, words * 4, hipHostMallocDefault) == hipSuccess &&
              hipMalloc((void**)&d->dev, bytes) == hipSuccess && hipMalloc(&d->ver, words * 4) == hipSuccess;
    if (ok) {
      s.pk = d->host;
      s.sig = d->host + cap * 32;
      s.off = reinterpret_cast<uint32_t*>(d->host + cap * 96);
      s.msg = d->host + d->msg_at;
      d->pk = d->dev;
      d->sig = d->dev + cap * 32;
      d->off = d->dev + cap * 96;
      d->msg = d->dev + d->msg_at;
    }
    ok = ok && hipEventCreateWithFlags(&d->uploaded, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&d->verified, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&d->done, hipEventDisableTiming) == hipSuccess;
    return ok ? AT2V_OK : AT2V_E_OOM;
  }
  void release(at2v::QueueSlot& s) {
    if (cpu_only) {
      std::free(s.verdicts);
      DevSlot* d = static_cast<DevSlot*>(s.backend);
      if (d) std::free(d->host);
      delete d;
      s.backend = nullptr;
      s.pk = s.sig = s.msg = nullptr;
      s.off = s.verdicts = nullptr;
      return;
    }
    const DeviceScope scope(device);
    if (s.verdicts) (void)hipHostFree(s.verdicts);
    s.pk = s.sig = s.msg = nullptr;
    s.off = s.verdicts = nullptr;
    DevSlot* d = static_cast<DevSlot*>(s.backend);
    if (!d) return;
    if (d->host) (void)hipHostFree(d->host);
    for (void* p : {(void*)d->dev, d->ver})
      if (p) (void)hipFree(p);
    for (hipEvent_t e : {d->uploaded, d->verified, d->done})
      if (e) (void)hipEventDestroy(e);
    delete d;
    s.backend = nullptr;
  }
  // H2D on h2d -> verify on comp[k % 2] (waits for its upload), verdict words written to pinned host memory (or a D2H
  // copy on the same comp stream with AT2V_QUEUE_DIRECT=0)
  // the slot's records on the CPU backend (cpu_ctx for a fallback), verdicts into its host words
  int verify_on_cpu(at2v::QueueSlot& s, at2v_ctx* c) {
    return at2v_verify_batch(c, s.pk, s.sig, s.msg, s.off, s.n, s.verdicts);
  }
  // a batch the device failed: drain what the slot's stream may still write into its verdict words, then the CPU
  int fall_back(at2v::QueueSlot& s, int rc) {
    DevSlot* d = static_cast<DevSlot*>(s.backend);
    if (!cpu_ctx) return rc;
    {
      const DeviceScope scope(device);
      if (d->stream) (void)hipStreamSynchronize(d->stream);
    }
    d->cpu_done = true;
    fallbacks.fetch_add(1, std::memory_order_relaxed);
    return verify_on_cpu(s, cpu_ctx);
  }
  int launch(at2v::QueueSlot& s) {
    DevSlot* d = static_cast<DevSlot*>(s.backend);
    d->cpu_done = false;
    if (cpu_only) return verify_on_cpu(s, ctx);
    const int rc = launch_gpu(s);
    return rc == AT2V_OK ? rc : fall_back(s, rc);
  }
  int launch_gpu(at2v::QueueSlot& s) {
    DevSlot* d = static_cast<DevSlot*>(s.backend);
    hipStream_t comp = this->comp[ncomp == 2 ? (launches++ & 1) : 0];
    d->stream = comp;
    const DeviceScope scope(device);
    hipError_t e = scope.err;
    const size_t n = s.n, words = (n + 31) / 32;
    if (n <= zerocopy_max) {  // the kernel reads the pinned host buffers (same layout) directly
      uint32_t* ver = direct ? s.verdicts : (uint32_t*)d->ver;
      if (e != hipSuccess) return AT2V_E_HIP;
      const int rc = at2v_verify_batch_device(ctx, s.pk, s.sig, s.msg, s.msg_used, s.off, n, ver, comp);
      if (rc) return rc;
      if (!direct) e = hipMemcpyAsync(s.verdicts, d->ver, words * 4, hipMemcpyDeviceToHost, comp);
      if (e == hipSuccess) e = hipEventRecord(d->done, comp);
      return e == hipSuccess ? AT2V_OK : AT2V_E_HIP;
    }
    if (!h2d && hipStreamCreateWithFlags(&h2d, hipStreamNonBlocking) != hipSuccess) return AT2V_E_HIP;
    if (d->msg_at + s.msg_used <= kSingleCopyMax) {  // one copy of the whole used span (small slots / latency mode)
      if (e == hipSuccess) e = hipMemcpyAsync(d->dev, d->host, d->msg_at + s.msg_used, hipMemcpyHostToDevice, h2d);
    } else {
      if (e == hipSuccess) e = hipMemcpyAsync(d->pk, s.pk, n * 32, hipMemcpyHostToDevice, h2d);
      if (e == hipSuccess) e = hipMemcpyAsync(d->sig, s.sig, n * 64, hipMemcpyHostToDevice, h2d);
      if (e == hipSuccess && s.msg_used) e = hipMemcpyAsync(d->msg, s.msg, s.msg_used, hipMemcpyHostToDevice, h2d);
      if (e == hipSuccess) e = hipMemcpyAsync(d->off, s.off, (n + 1) * 4, hipMemcpyHostToDevice, h2d);
    }
    if (e == hipSuccess) e = hipEventRecord(d->uploaded, h2d);
    if (e == hipSuccess) e = hipStreamWaitEvent(comp, d->uploaded, 0);
    if (e != hipSuccess) return AT2V_E_HIP;
    uint32_t* ver = direct ? s.verdicts : (uint32_t*)d->ver;
    const int rc = at2v_verify_batch_device(ctx, (const uint8_t*)d->pk, (const uint8_t*)d->sig, (const uint8_t*)d->msg,
                                            s.msg_used, (const uint32_t*)d->off, n, ver, comp);
    if (rc) return rc;
    if (!direct) e = hipMemcpyAsync(s.verdicts, d->ver, words * 4, hipMemcpyDeviceToHost, comp);
    if (e == hipSuccess) e = hipEventRecord(d->done, comp);
    return e == hipSuccess ? AT2V_OK : AT2V_E_HIP;
  }
  int wait(at2v::QueueSlot& s) {
    DevSlot* d = static_cast<DevSlot*>(s.backend);
    if (cpu_only || d->cpu_done) return AT2V_OK;  // verified in launch()
    const int rc = wait_gpu(d);
    return rc == AT2V_OK ? rc : fall_back(s, rc);
  }
  int wait_gpu(DevSlot* d) {
    if (spin_us) {
      const auto t0 = std::chrono::steady_clock::now();
      for (unsigned k = 0;; ++k) {
        const hipError_t q = hipEventQuery(d->done);
        if (q == hipSuccess) return AT2V_OK;
        if (q != hipErrorNotReady) return AT2V_E_HIP;
        if ((k & 63) == 63 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us))
          break;
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      }
    }
    return hipEventSynchronize(d->done) == hipSuccess ? AT2V_OK : AT2V_E_HIP;
  }
};

}  // namespace

struct at2v_queue {
  HipBackend be;
  at2v::BatchQueue<HipBackend>* q = nullptr;
};

struct at2v_ledger {
  at2v::Ledger l;
};

extern "C" {

int at2v_queue_create(const at2v_queue_opts* opts, at2v_queue** out) {
  if (!out) return AT2V_E_INVALID;
  *out = nullptr;
  at2v_queue_opts o{0, AT2V_POLICY_DALEK_V1, 0, 0, 0, 0, 0, 0, 0};
  if (opts) o = *opts;
  at2v::QueueOpts qo;
  if (o.max_batch) qo.max_batch = o.max_batch;
  if (o.max_delay_us) qo.max_delay_us = o.max_delay_us;
  if (o.max_msg_bytes) qo.max_msg_bytes = o.max_msg_bytes;
  if (o.depth) qo.depth = (int)o.depth;
  qo.eager = (o.flags & AT2V_QUEUE_EAGER) != 0;
  if (const char* v = at2v::test_env("AT2V_QUEUE_LAUNCH_HERE")) qo.launch_here = std::atoi(v) != 0;  // (A/B)
  if (o.flags & ~(AT2V_QUEUE_EAGER | AT2V_QUEUE_SENDER_COMB | AT2V_QUEUE_CPU | AT2V_QUEUE_CPU_FALLBACK))
    return AT2V_E_INVALID;
  if ((o.flags & AT2V_QUEUE_CPU) && (o.flags & (AT2V_QUEUE_SENDER_COMB | AT2V_QUEUE_CPU_FALLBACK))) return AT2V_E_INVALID;
  if (qo.depth < 2 || qo.max_batch >= (1u << 31) || (uint64_t)qo.max_batch * qo.max_msg_bytes >= (1ull << 32))
    return AT2V_E_INVALID;
  at2v_queue* q = new (std::nothrow) at2v_queue;
  if (!q) return AT2V_E_OOM;
  int rc = q->be.init(o);
  if (rc == AT2V_OK) {
    q->q = new (std::nothrow) at2v::BatchQueue<HipBackend>(q->be, qo);
    rc = q->q ? q->q->start() : AT2V_E_OOM;
  }
  if (rc != AT2V_OK) {
    at2v_queue_destroy(q);
    return rc < 0 ? rc : AT2V_E_HIP;
  }
  *out = q;
  return AT2V_OK;
}

void at2v_queue_destroy(at2v_queue* q) {
  if (!q) return;
  delete q->q;  // stop(): seal, complete, join, free the slots
  q->be.fini();
  delete q;
}

int at2v_queue_submit(at2v_queue* q, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                      const uint32_t* msg_off, size_t n, uint64_t* first_ticket) {
  if (!q || !q->q) return AT2V_E_INVALID;
  if (n == 0) return AT2V_OK;
  if (!pk || !sig || !msg_off || (!msg && msg_off[n] != msg_off[0])) return AT2V_E_INVALID;
  return q->q->submit(pk, sig, msg, msg_off, n, first_ticket) == 0 ? AT2V_OK : AT2V_E_INVALID;
}

int at2v_queue_flush(at2v_queue* q) {
  if (!q || !q->q) return AT2V_E_INVALID;
  q->q->flush();
  return AT2V_OK;
}

long at2v_queue_poll(at2v_queue* q, uint64_t* tickets, uint8_t* verdicts, size_t max, uint32_t timeout_us) {
  if (!q || !q->q || (max && (!tickets || !verdicts))) return AT2V_E_INVALID;
  return q->q->poll(tickets, verdicts, max, timeout_us);
}

int at2v_queue_get_stats(at2v_queue* q, at2v_queue_stats* out) {
  if (!q || !q->q || !out) return AT2V_E_INVALID;
  const at2v::QueueStats s = q->q->stats();
  out->submitted = s.submitted;
  out->completed = s.completed;
  out->batches = s.batches;
  out->failed_batches = s.failed_batches;
  out->mean_batch = s.mean_batch;
  out->p50_us = s.p50_us;
  out->p99_us = s.p99_us;
  out->max_us = s.max_us;
  out->cpu_fallbacks = q->be.fallbacks.load(std::memory_order_relaxed);
  return AT2V_OK;
}

int at2v_queue_reset_latency(at2v_queue* q) {
  if (!q || !q->q) return AT2V_E_INVALID;
  q->q->reset_latency();
  return AT2V_OK;
}

long at2v_pack_send_asset(const at2v_send_asset_request* req, size_t n, int wire, uint8_t* pk_out, uint8_t* sig_out,
                          uint8_t* msg_out, uint32_t* msg_off_out, uint8_t* recipient_out, uint8_t* status_out) {
  if (n && (!req || !pk_out || !sig_out || !msg_out || !msg_off_out || !recipient_out || !status_out))
    return AT2V_E_INVALID;
  if (wire != AT2V_WIRE_BYTES && wire != AT2V_WIRE_ARRAY) return AT2V_E_INVALID;
  if (!msg_off_out) return AT2V_E_INVALID;
  long ok = 0;
  uint32_t o = 0;
  msg_off_out[0] = 0;
  for (size_t i = 0; i < n; ++i) {
    const at2v_send_asset_request& r = req[i];
    // rpc.rs order: recipient (:265), sender (:269), signature (:281)
    const uint8_t* rcp = at2v::wire_field(r.recipient, r.recipient_len, 32, wire);
    const uint8_t* snd = rcp ? at2v::wire_field(r.sender, r.sender_len, 32, wire) : nullptr;
    const uint8_t* sg = snd ? at2v::wire_field(r.signature, r.signature_len, 64, wire) : nullptr;
    const uint8_t st = !rcp ? AT2V_PACK_BAD_RECIPIENT : !snd ? AT2V_PACK_BAD_SENDER : !sg ? AT2V_PACK_BAD_SIGNATURE
                                                                                           : AT2V_PACK_OK;
    status_out[i] = st;
    if (st == AT2V_PACK_OK) {
      std::memcpy(pk_out + 32 * i, snd, 32);
      std::memcpy(sig_out + 64 * i, sg, 64);
      std::memcpy(recipient_out + 32 * i, rcp, 32);
      o += (uint32_t)at2v::thin_transaction(msg_out + o, rcp, r.amount, wire);
      ++ok;
    } else {
      std::memset(pk_out + 32 * i, 0, 32);
      std::memset(sig_out + 64 * i, 0, 64);
      std::memset(recipient_out + 32 * i, 0, 32);
    }
    msg_off_out[i + 1] = o;
  }
  return ok;
}

int at2v_ledger_create(at2v_ledger** out) {
  if (!out) return AT2V_E_INVALID;
  *out = new (std::nothrow) at2v_ledger;
  return *out ? AT2V_OK : AT2V_E_OOM;
}

void at2v_ledger_destroy(at2v_ledger* l) { delete l; }

int at2v_ledger_balance(const at2v_ledger* l, const uint8_t pk[32], uint64_t* out) {
  if (!l || !pk || !out) return AT2V_E_INVALID;
  *out = l->l.balance(at2v::make_key(pk));
  return AT2V_OK;
}

int at2v_ledger_last_sequence(const at2v_ledger* l, const uint8_t pk[32], uint32_t* out) {
  if (!l || !pk || !out) return AT2V_E_INVALID;
  *out = l->l.last_sequence(at2v::make_key(pk));
  return AT2V_OK;
}

int at2v_ledger_transfer(at2v_ledger* l, const uint8_t sender[32], uint32_t sequence, const uint8_t recipient[32],
                         uint64_t amount) {
  if (!l || !sender || !recipient) return AT2V_E_INVALID;
  return l->l.transfer(at2v::make_key(sender), sequence, at2v::make_key(recipient), amount);
}

int at2v_ledger_recent_put(at2v_ledger* l, const uint8_t sender[32], uint32_t sequence, const uint8_t recipient[32],
                           uint64_t amount, uint64_t now_us) {
  if (!l || !sender || !recipient) return AT2V_E_INVALID;
  l->l.recent_put(at2v::make_key(sender), sequence, at2v::make_key(recipient), amount, now_us);
  return AT2V_OK;
}

long at2v_ledger_recent_get(const at2v_ledger* l, at2v_full_transaction* out, size_t max) {
  if (!l || (max && !out)) return AT2V_E_INVALID;
  long k = 0;
  for (const auto& t : l->l.recent()) {
    if ((size_t)k == max) break;
    at2v_full_transaction& o = out[k++];
    o.timestamp_us = t.timestamp_us;
    std::memcpy(o.sender, t.sender.data(), 32);
    o.sender_sequence = t.sender_sequence;
    std::memcpy(o.recipient, t.recipient.data(), 32);
    o.amount = t.amount;
    o.state = t.state;
  }
  return k;
}

int at2v_ledger_deliver(at2v_ledger* l, const uint8_t* sender, const uint32_t* sequence, const uint8_t* recipient,
                        const uint64_t* amount, const uint32_t* verdicts, size_t n, uint64_t now_us,
                        at2v_apply_stats* stats) {
  if (!l || (n && (!sender || !sequence || !recipient || !amount))) return AT2V_E_INVALID;
  std::vector<at2v::Payload> batch;
  batch.reserve(n);
  uint64_t rejected = 0;
  for (size_t i = 0; i < n; ++i) {
    if (verdicts && !((verdicts[i >> 5] >> (i & 31)) & 1u)) {
      ++rejected;
      continue;
    }
    batch.push_back(at2v::Payload{sequence[i], at2v::make_key(sender + 32 * i), at2v::make_key(recipient + 32 * i),
                                  amount[i], now_us, 0});
  }
  at2v::ApplyStats st;
  st.rejected = rejected;
  l->l.deliver(batch, now_us, &st);
  if (stats) {
    stats->delivered = batch.size();
    stats->rejected = st.rejected;
    stats->applied = st.applied;
    stats->requeued = st.requeued;
    stats->expired = st.expired;
    stats->passes = st.passes;
  }
  return AT2V_OK;
}

long at2v_ledger_pending(const at2v_ledger* l) { return l ? (long)l->l.pending() : AT2V_E_INVALID; }

}  // extern "C"
