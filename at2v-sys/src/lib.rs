//! at2v-sys — raw bindings of `include/at2v.h` (libat2v: MI355X batch Ed25519 verification for at2-node)
//! plus a thin safe layer for the two call shapes the server needs.
//!
//! Where it plugs into the reference (/root/reference, at2-node v1):
//!   * per payload, as the body of drop's `Signature::verify` that sieve/murmur call for every payload
//!     broadcast at src/bin/server/rpc.rs:275-284 -> `verify_one` (CPU, reentrant);
//!   * per gossiped batch, ahead of `deliver()` at rpc.rs:156-173 -> `BatchVerifier::verify` (GPU, or the CPU
//!     backend on a node without one: `BatchVerifier::cpu`) or the ingest queue (`at2v_queue_*`);
//!   * one process per GPU: `at2v_comm_init_rank` + `at2v_verify_batch_sharded` (RCCL all-gather of the
//!     verdict bitmap over xGMI).
//! The extern block below must stay identical to include/at2v.h (names, argument counts, integer widths);
//! tests/test_sys_crate.py checks it, since this image cannot run cargo.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_long, c_void};

// ---------------------------------------------------------------- types and constants (at2v.h)

#[repr(C)]
pub struct At2vCtx {
    _private: [u8; 0],
}
#[repr(C)]
pub struct At2vQueue {
    _private: [u8; 0],
}
#[repr(C)]
pub struct At2vLedger {
    _private: [u8; 0],
}

/// include/at2v.h AT2V_ABI_VERSION: the layouts of the #[repr(C)] structs below. `BatchVerifier::new` and
/// `Queue::new` refuse a library that reports another version (the structs are copied whole by the library).
pub const AT2V_ABI_VERSION: c_int = 7;

pub const AT2V_POLICY_DALEK_V1: c_int = 0;
pub const AT2V_POLICY_LIBSODIUM_1_0_18: c_int = 1;

pub const AT2V_OK: c_int = 0;
pub const AT2V_E_INVALID: c_int = -1;
pub const AT2V_E_NODEVICE: c_int = -2;
pub const AT2V_E_HIP: c_int = -3;
pub const AT2V_E_OOM: c_int = -4;
pub const AT2V_E_ALIGN: c_int = -5;
pub const AT2V_E_RCCL: c_int = -6;
pub const AT2V_E_PEER: c_int = -7;

pub const AT2V_UNIQUE_ID_BYTES: usize = 128;

pub const AT2V_WIRE_BYTES: c_int = 0;
pub const AT2V_WIRE_ARRAY: c_int = 1;
pub const AT2V_PACK_OK: u8 = 0;
pub const AT2V_PACK_BAD_RECIPIENT: u8 = 1;
pub const AT2V_PACK_BAD_SENDER: u8 = 2;
pub const AT2V_PACK_BAD_SIGNATURE: u8 = 3;

pub const AT2V_TX_OK: c_int = 0;
pub const AT2V_TX_INCONSECUTIVE_SEQUENCE: c_int = 1;
pub const AT2V_TX_OVERFLOW: c_int = 2;
pub const AT2V_TX_UNDERFLOW: c_int = 3;
pub const AT2V_TX_PENDING: i32 = 0;
pub const AT2V_TX_SUCCESS: i32 = 1;
pub const AT2V_TX_FAILURE: i32 = 2;

/// at2v_queue_poll verdict bytes
pub const AT2V_VERDICT_INVALID: u8 = 0;
pub const AT2V_VERDICT_VALID: u8 = 1;
pub const AT2V_VERDICT_FAILED: u8 = 0xff;

/// `Default`: device 0, one GPU, DALEK_V1, library-default small-batch threshold, no sender cache, no CPU fallback.
/// (Not derived: `num_gpus = 0` selects the CPU batch backend since ABI version 6.)
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct At2vOpts {
    pub device: c_int,
    /// devices `device..device+num_gpus-1`; 0 = the CPU batch backend (no device, `cpu_threads` host threads)
    pub num_gpus: c_int,
    pub policy: c_int,
    /// launches of at most this many records run the low-latency kernel; 0 = 32768, AT2V_SMALL_BATCH_OFF = never
    pub small_batch_max: u32,
    /// per-sender A cache capacity in distinct public keys; 0 = off
    pub sender_cache: u32,
    /// with sender_cache: 1 = per-key combs (all-hit chunks verify by table additions only); 0 = off
    pub sender_comb: u32,
    /// host threads of the CPU backend (num_gpus = 0, or AT2V_CTX_CPU_FALLBACK); 0 = every usable CPU
    pub cpu_threads: u32,
    /// AT2V_CTX_CPU_FALLBACK | AT2V_CTX_ADMIT_FIRST | AT2V_CTX_BCOMB_WIDE
    pub flags: u32,
}

impl Default for At2vOpts {
    fn default() -> Self {
        At2vOpts { device: 0, num_gpus: 1, policy: AT2V_POLICY_DALEK_V1, small_batch_max: 0, sender_cache: 0,
                   sender_comb: 0, cpu_threads: 0, flags: 0 }
    }
}

/// `At2vOpts::flags`: a GPU context re-runs a failed host-buffer batch on the CPU backend (same verdicts).
pub const AT2V_CTX_CPU_FALLBACK: u32 = 1;
/// `At2vOpts::flags`: sender-cache keys claim a payload at their first sighting (default: the second).
pub const AT2V_CTX_ADMIT_FIRST: u32 = 2;
/// `At2vOpts::flags`: with sender_comb, the throughput kernel's comb of B with 24-bit windows (11.8 GB, default 20-bit).
pub const AT2V_CTX_BCOMB_WIDE: u32 = 4;

/// `At2vInfo::experiments` bits: timing-only builds with wrong verdicts (at2v_create refuses them unless
/// AT2V_ALLOW_EXPERIMENT=1 is set in the process environment)
pub const AT2V_EXPERIMENT_TAB128: u32 = 1;
pub const AT2V_EXPERIMENT_COMB_HOT: u32 = 2;
pub const AT2V_EXPERIMENT_SLOT_WAVES: u32 = 4;
pub const AT2V_EXPERIMENT_CONST_MSG: u32 = 8;
pub const AT2V_EXPERIMENT_BCOMB_NOBUILD: u32 = 16;
pub const AT2V_EXPERIMENT_COMB3: u32 = 32;

pub const AT2V_SMALL_BATCH_DEFAULT: u32 = 32768;
pub const AT2V_SMALL_BATCH_OFF: u32 = 0xffffffff;

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct At2vInfo {
    pub num_gpus: c_int,
    pub grid_blocks: c_int,
    pub block_threads: c_int,
    pub waves_per_cu: c_int,
    pub cus: c_int,
    pub vgprs: c_int,
    pub rank: c_int,
    pub world: c_int,
    pub gathers: u64,
    pub cache_entries: u64,
    pub cache_chunks: u64,
    pub cache_chunk_hits: u64,
    pub cache_capacity: u64,
    pub cache_claims: u64,
    pub cache_evicted: u64,
    pub cache_compactions: u64,
    pub cpu_threads: u64,
    pub cpu_batches: u64,
    pub cpu_fallbacks: u64,
    pub cache_sightings: u64,
    pub cache_built: u64,
    pub cache_build_us: u64,
    pub cache_record_hits: u64,
    /// AT2V_EXPERIMENT_* bits compiled into the library (0 in a shipped build)
    pub experiments: u64,
    /// chunks staged by the host-buffer calls' pipeline
    pub host_chunks: u64,
}

/// `Default`: device 0, DALEK_V1, and the library defaults for every size (65536 records, 1 ms, 256 B, depth 3).
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct At2vQueueOpts {
    pub device: c_int,
    pub policy: c_int,
    pub max_batch: u32,
    pub max_delay_us: u32,
    pub max_msg_bytes: u32,
    pub depth: u32,
    pub flags: u32,
    /// with AT2V_QUEUE_SENDER_COMB: keys the queue's context caches (HBM per key: see include/at2v.h); 0 = 1024
    pub sender_cache: u32,
    /// AT2V_QUEUE_CPU / AT2V_QUEUE_CPU_FALLBACK: host threads (0 = every usable CPU)
    pub cpu_threads: u32,
}

/// `At2vQueueOpts::flags`: also seal the filling batch whenever no batch is in flight (latency mode).
pub const AT2V_QUEUE_EAGER: u32 = 1;
pub const AT2V_QUEUE_SENDER_COMB: u32 = 2;
/// `At2vQueueOpts::flags`: batches verified by the CPU backend (no device).
pub const AT2V_QUEUE_CPU: u32 = 4;
/// `At2vQueueOpts::flags`: a batch the device fails is verified on the CPU backend instead.
pub const AT2V_QUEUE_CPU_FALLBACK: u32 = 8;

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct At2vQueueStats {
    pub submitted: u64,
    pub completed: u64,
    pub batches: u64,
    pub failed_batches: u64,
    pub mean_batch: f64,
    pub p50_us: f64,
    pub p99_us: f64,
    pub max_us: f64,
    pub cpu_fallbacks: u64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct At2vSendAssetRequest {
    pub sender: *const u8,
    pub sender_len: usize,
    pub sequence: u32,
    pub recipient: *const u8,
    pub recipient_len: usize,
    pub amount: u64,
    pub signature: *const u8,
    pub signature_len: usize,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct At2vFullTransaction {
    pub timestamp_us: u64,
    pub sender: [u8; 32],
    pub sender_sequence: u32,
    pub recipient: [u8; 32],
    pub amount: u64,
    pub state: i32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct At2vApplyStats {
    pub delivered: u64,
    pub rejected: u64,
    pub applied: u64,
    pub requeued: u64,
    pub expired: u64,
    pub passes: u64,
}

// ---------------------------------------------------------------- functions (at2v.h, same order)

extern "C" {
    pub fn at2v_abi_version() -> c_int;
    pub fn at2v_create(opts: *const At2vOpts, out: *mut *mut At2vCtx) -> c_int;
    pub fn at2v_destroy(ctx: *mut At2vCtx);
    pub fn at2v_verify_batch(ctx: *mut At2vCtx, pk: *const u8, sig: *const u8, msg: *const u8, msg_off: *const u32,
                             n: usize, verdicts: *mut u32) -> c_int;
    pub fn at2v_verify_batch_submit(ctx: *mut At2vCtx, pk: *const u8, sig: *const u8, msg: *const u8,
                                    msg_off: *const u32, n: usize, verdicts: *mut u32, ticket: *mut u64) -> c_int;
    pub fn at2v_verify_batch_wait(ctx: *mut At2vCtx, ticket: u64) -> c_int;
    pub fn at2v_verify_batch_device(ctx: *mut At2vCtx, d_pk: *const u8, d_sig: *const u8, d_msg: *const u8,
                                    msg_bytes: usize, d_msg_off: *const u32, n: usize, d_verdicts: *mut u32,
                                    hip_stream: *mut c_void) -> c_int;
    pub fn at2v_verify_one(pk: *const u8, sig: *const u8, msg: *const u8, len: usize) -> c_int;
    pub fn at2v_verify_one_policy(pk: *const u8, sig: *const u8, msg: *const u8, len: usize, policy: c_int) -> c_int;
    pub fn at2v_strerror(code: c_int) -> *const c_char;
    pub fn at2v_gen_records_device(ctx: *mut At2vCtx, cfg_seed: u64, first: u64, n: usize, msg_len: u32,
                                   d_pk: *mut u8, d_sig: *mut u8, d_msg: *mut u8, d_msg_off: *mut u32,
                                   hip_stream: *mut c_void) -> c_int;
    pub fn at2v_gen_records_senders_device(ctx: *mut At2vCtx, cfg_seed: u64, first: u64, n: usize, msg_len: u32,
                                           senders: u64, d_pk: *mut u8, d_sig: *mut u8, d_msg: *mut u8,
                                           d_msg_off: *mut u32, hip_stream: *mut c_void) -> c_int;
    pub fn at2v_gen_records_keys_device(ctx: *mut At2vCtx, cfg_seed: u64, first: u64, n: usize, msg_len: u32,
                                        d_keys: *const u64, d_pk: *mut u8, d_sig: *mut u8, d_msg: *mut u8,
                                        d_msg_off: *mut u32, hip_stream: *mut c_void) -> c_int;
    pub fn at2v_sign_batch(ctx: *mut At2vCtx, seeds: *const u8, msg: *const u8, msg_off: *const u32, n: usize,
                           pk_out: *mut u8, sig_out: *mut u8) -> c_int;
    pub fn at2v_get_info(ctx: *mut At2vCtx, out: *mut At2vInfo) -> c_int;

    pub fn at2v_comm_get_unique_id(out: *mut u8) -> c_int;
    pub fn at2v_comm_init_rank(ctx: *mut At2vCtx, unique_id: *const u8, rank: c_int, world: c_int) -> c_int;
    pub fn at2v_verify_shard_gather_device(ctx: *mut At2vCtx, d_pk: *const u8, d_sig: *const u8, d_msg: *const u8,
                                           msg_bytes: usize, d_msg_off: *const u32, n_local: usize,
                                           words_per_rank: usize, d_bitmap: *mut u32, hip_stream: *mut c_void)
                                           -> c_int;
    pub fn at2v_verify_batch_sharded(ctx: *mut At2vCtx, pk: *const u8, sig: *const u8, msg: *const u8,
                                     msg_off: *const u32, n: usize, verdicts: *mut u32) -> c_int;

    pub fn at2v_queue_create(opts: *const At2vQueueOpts, out: *mut *mut At2vQueue) -> c_int;
    pub fn at2v_queue_destroy(q: *mut At2vQueue);
    pub fn at2v_queue_submit(q: *mut At2vQueue, pk: *const u8, sig: *const u8, msg: *const u8, msg_off: *const u32,
                             n: usize, first_ticket: *mut u64) -> c_int;
    pub fn at2v_queue_flush(q: *mut At2vQueue) -> c_int;
    pub fn at2v_queue_poll(q: *mut At2vQueue, tickets: *mut u64, verdicts: *mut u8, max: usize, timeout_us: u32)
                           -> c_long;
    pub fn at2v_queue_get_stats(q: *mut At2vQueue, out: *mut At2vQueueStats) -> c_int;
    pub fn at2v_queue_reset_latency(q: *mut At2vQueue) -> c_int;

    pub fn at2v_pack_send_asset(req: *const At2vSendAssetRequest, n: usize, wire: c_int, pk_out: *mut u8,
                                sig_out: *mut u8, msg_out: *mut u8, msg_off_out: *mut u32, recipient_out: *mut u8,
                                status_out: *mut u8) -> c_long;
    pub fn at2v_decode_points(ctx: *mut At2vCtx, pts: *const u8, n: usize, valid_words: *mut u32) -> c_int;

    pub fn at2v_ledger_create(out: *mut *mut At2vLedger) -> c_int;
    pub fn at2v_ledger_destroy(l: *mut At2vLedger);
    pub fn at2v_ledger_balance(l: *const At2vLedger, pk: *const u8, out: *mut u64) -> c_int;
    pub fn at2v_ledger_last_sequence(l: *const At2vLedger, pk: *const u8, out: *mut u32) -> c_int;
    pub fn at2v_ledger_transfer(l: *mut At2vLedger, sender: *const u8, sequence: u32, recipient: *const u8,
                                amount: u64) -> c_int;
    pub fn at2v_ledger_recent_put(l: *mut At2vLedger, sender: *const u8, sequence: u32, recipient: *const u8,
                                  amount: u64, now_us: u64) -> c_int;
    pub fn at2v_ledger_recent_get(l: *const At2vLedger, out: *mut At2vFullTransaction, max: usize) -> c_long;
    pub fn at2v_ledger_deliver(l: *mut At2vLedger, sender: *const u8, sequence: *const u32, recipient: *const u8,
                               amount: *const u64, verdicts: *const u32, n: usize, now_us: u64,
                               stats: *mut At2vApplyStats) -> c_int;
    pub fn at2v_ledger_pending(l: *const At2vLedger) -> c_long;
}

// ---------------------------------------------------------------- safe layer

/// A negative at2v return code (backend failure: no device, HIP, OOM, RCCL). Never "invalid signature".
#[derive(Debug, Clone, Copy, PartialEq, Eq)]
pub struct Error(pub c_int);

impl std::fmt::Display for Error {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        let s = unsafe { std::ffi::CStr::from_ptr(at2v_strerror(self.0)) };
        write!(f, "at2v error {}: {}", self.0, s.to_string_lossy())
    }
}

impl std::error::Error for Error {}

fn check(rc: c_int) -> Result<c_int, Error> {
    if rc < 0 {
        Err(Error(rc))
    } else {
        Ok(rc)
    }
}

/// One signature on the CPU, dalek-1.x semantics: the body of drop's per-payload `Signature::verify`.
/// Reentrant; needs no GPU.
pub fn verify_one(public_key: &[u8; 32], signature: &[u8; 64], message: &[u8]) -> Result<bool, Error> {
    let m = if message.is_empty() { std::ptr::null() } else { message.as_ptr() };
    check(unsafe { at2v_verify_one(public_key.as_ptr(), signature.as_ptr(), m, message.len()) }).map(|v| v == 1)
}

/// The C side copies message bytes up to `msg_off[n]` and takes no length: a safe wrapper must prove every offset is in
/// `msg` and non-decreasing before it hands the pointers over.
fn check_records(pk: &[u8], sig: &[u8], msg: &[u8], msg_off: &[u32]) -> Result<usize, Error> {
    let n = msg_off.len().saturating_sub(1);
    if pk.len() != 32 * n || sig.len() != 64 * n {
        return Err(Error(AT2V_E_INVALID));
    }
    if msg_off.windows(2).any(|w| w[1] < w[0]) || msg_off.last().map_or(false, |&e| e as usize > msg.len()) {
        return Err(Error(AT2V_E_INVALID));
    }
    Ok(n)
}

fn check_abi() -> Result<(), Error> {
    if unsafe { at2v_abi_version() } != AT2V_ABI_VERSION {
        return Err(Error(AT2V_E_INVALID));
    }
    Ok(())
}

/// Owner of an at2v context (GPUs, or the CPU backend). Not Sync: one thread at a time; call from `spawn_blocking` or
/// a dedicated thread, never on an async executor thread.
pub struct BatchVerifier(*mut At2vCtx);

unsafe impl Send for BatchVerifier {}

impl BatchVerifier {
    pub fn new(opts: &At2vOpts) -> Result<Self, Error> {
        check_abi()?;
        let mut p = std::ptr::null_mut();
        check(unsafe { at2v_create(opts, &mut p) })?;
        Ok(BatchVerifier(p))
    }

    /// `num_gpus` devices from `device` on, library defaults otherwise.
    pub fn on_devices(device: i32, num_gpus: i32, policy: c_int) -> Result<Self, Error> {
        Self::new(&At2vOpts { device, num_gpus, policy, ..Default::default() })
    }

    /// The CPU batch backend (a node without a gfx950): `cpu_threads` host threads (0 = every usable CPU) over the
    /// kernels' own verify routine; the drop-in for the reference's `num_cpus::get()` verify workers (rpc.rs:124-125).
    pub fn cpu(cpu_threads: u32, policy: c_int) -> Result<Self, Error> {
        Self::new(&At2vOpts { num_gpus: 0, policy, cpu_threads, ..Default::default() })
    }

    /// One process per GPU: join the node's RCCL communicator (collective over `world` ranks).
    pub fn init_rank(&mut self, unique_id: &[u8; AT2V_UNIQUE_ID_BYTES], rank: i32, world: i32) -> Result<(), Error> {
        check(unsafe { at2v_comm_init_rank(self.0, unique_id.as_ptr(), rank, world) }).map(|_| ())
    }

    /// Records in the at2v_verify_batch layout -> one bool per record (bit i of the verdict bitmap).
    /// `sharded`: every rank passes the same node batch; each verifies its range and the RCCL all-gather
    /// returns the whole bitmap (requires `init_rank`). Err(AT2V_E_PEER): another rank failed; discard the batch.
    pub fn verify(&mut self, pk: &[u8], sig: &[u8], msg: &[u8], msg_off: &[u32], sharded: bool)
                  -> Result<Vec<bool>, Error> {
        let n = check_records(pk, sig, msg, msg_off)?;
        let mut words = vec![0u32; (n + 31) / 32];
        let m = if msg.is_empty() { std::ptr::null() } else { msg.as_ptr() };
        let rc = unsafe {
            if sharded {
                at2v_verify_batch_sharded(self.0, pk.as_ptr(), sig.as_ptr(), m, msg_off.as_ptr(), n,
                                          words.as_mut_ptr())
            } else {
                at2v_verify_batch(self.0, pk.as_ptr(), sig.as_ptr(), m, msg_off.as_ptr(), n, words.as_mut_ptr())
            }
        };
        check(rc)?;
        Ok((0..n).map(|i| (words[i / 32] >> (i % 32)) & 1 == 1).collect())
    }

    /// Device-resident records (the layout of `verify`, in HBM of the context's first device), asynchronous on
    /// `hip_stream` (a hipStream_t; null = the null stream): the verdict words are valid once the stream has
    /// reached this point.
    ///
    /// # Safety
    /// Every pointer must be a device allocation of the context's device with the sizes of include/at2v.h
    /// (`d_pk` n x 32 B and `d_sig` n x 64 B, 16-byte aligned; `d_msg_off` n + 1 offsets into `msg_bytes` bytes at
    /// `d_msg`; `d_verdicts` ceil(n/32) words) and stay alive until the stream has passed the launch.
    pub unsafe fn verify_device(&mut self, d_pk: *const u8, d_sig: *const u8, d_msg: *const u8, msg_bytes: usize,
                                d_msg_off: *const u32, n: usize, d_verdicts: *mut u32, hip_stream: *mut c_void)
                                -> Result<(), Error> {
        check(at2v_verify_batch_device(self.0, d_pk, d_sig, d_msg, msg_bytes, d_msg_off, n, d_verdicts, hip_stream))
            .map(|_| ())
    }

    pub fn info(&self) -> Result<At2vInfo, Error> {
        let mut i = At2vInfo::default();
        check(unsafe { at2v_get_info(self.0, &mut i) })?;
        Ok(i)
    }
}

impl Drop for BatchVerifier {
    fn drop(&mut self) {
        unsafe { at2v_destroy(self.0) }
    }
}

/// The server's verify call site: payloads go in with `submit`, verdicts come back from `poll`
/// in submission (ticket) order. Thread-safe on the library side (any number of producers, poll from any thread).
pub struct Queue(*mut At2vQueue);

unsafe impl Send for Queue {}
unsafe impl Sync for Queue {}

/// One polled verdict: `Some(true)` valid, `Some(false)` invalid, `None` the batch failed on the device
/// (re-submit; it is neither valid nor invalid).
pub type Verdict = Option<bool>;

impl Queue {
    pub fn new(opts: &At2vQueueOpts) -> Result<Self, Error> {
        check_abi()?;
        let mut p = std::ptr::null_mut();
        check(unsafe { at2v_queue_create(opts, &mut p) })?;
        Ok(Queue(p))
    }

    /// Records in the at2v_verify_batch layout; returns the ticket of the first (the rest follow consecutively).
    /// Blocks only while every batch slot is in flight (backpressure).
    pub fn submit(&self, pk: &[u8], sig: &[u8], msg: &[u8], msg_off: &[u32]) -> Result<u64, Error> {
        let n = check_records(pk, sig, msg, msg_off)?;
        let m = if msg.is_empty() { std::ptr::null() } else { msg.as_ptr() };
        let mut first = 0u64;
        check(unsafe { at2v_queue_submit(self.0, pk.as_ptr(), sig.as_ptr(), m, msg_off.as_ptr(), n, &mut first) })?;
        Ok(first)
    }

    pub fn flush(&self) -> Result<(), Error> {
        check(unsafe { at2v_queue_flush(self.0) }).map(|_| ())
    }

    /// Up to `max` completed (ticket, verdict) pairs in ticket order, waiting up to `timeout_us` for the first.
    pub fn poll(&self, max: usize, timeout_us: u32) -> Result<Vec<(u64, Verdict)>, Error> {
        let mut t = vec![0u64; max];
        let mut v = vec![0u8; max];
        let k = unsafe { at2v_queue_poll(self.0, t.as_mut_ptr(), v.as_mut_ptr(), max, timeout_us) };
        if k < 0 {
            return Err(Error(k as c_int));
        }
        Ok((0..k as usize)
            .map(|i| (t[i], match v[i] { AT2V_VERDICT_VALID => Some(true), AT2V_VERDICT_INVALID => Some(false), _ => None }))
            .collect())
    }

    pub fn stats(&self) -> Result<At2vQueueStats, Error> {
        let mut s = At2vQueueStats::default();
        check(unsafe { at2v_queue_get_stats(self.0, &mut s) })?;
        Ok(s)
    }
}

impl Drop for Queue {
    /// Seals and completes everything submitted, then frees.
    fn drop(&mut self) {
        unsafe { at2v_queue_destroy(self.0) }
    }
}

/// RCCL unique id for `BatchVerifier::init_rank` (rank 0 creates it and sends it to the others).
pub fn unique_id() -> Result<[u8; AT2V_UNIQUE_ID_BYTES], Error> {
    let mut id = [0u8; AT2V_UNIQUE_ID_BYTES];
    check(unsafe { at2v_comm_get_unique_id(id.as_mut_ptr()) })?;
    Ok(id)
}

#[cfg(test)]
mod tests {
    use super::*;

    /// an offset array that runs past `msg` (or goes backwards) must be refused by the safe layer before any
    /// pointer reaches the C side, which reads message bytes up to `msg_off[n]` without a length.
    #[test]
    fn safe_layer_rejects_offsets_outside_msg() {
        let (pk, sig, msg) = ([0u8; 32], [0u8; 64], [0u8; 4]);
        assert!(check_records(&pk, &sig, &msg, &[0, 4]).is_ok());
        assert!(check_records(&pk, &sig, &msg, &[0, 5]).is_err()); // past the end of msg
        assert!(check_records(&pk, &sig, &msg, &[3, 2]).is_err()); // decreasing
        assert!(check_records(&pk, &sig[..32], &msg, &[0, 4]).is_err()); // short signature
        assert!(check_records(&[], &[], &[], &[]).is_ok()); // an empty batch
    }
}
