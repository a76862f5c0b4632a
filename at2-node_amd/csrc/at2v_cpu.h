// at2v_cpu.h — the CPU batch backend of the product (at2v_opts.num_gpus = 0, and the opt-in fallback of a GPU context,
// AT2V_CTX_CPU_FALLBACK). It replaces the reference's SystemManager::run(.., num_cpus::get()) workers, which verify one
// payload each (/root/reference/src/bin/server/rpc.rs:124-125, the per-payload drop::crypto::sign check behind
// rpc.rs:275-284), with a pool of host threads over the SAME verify routine the GPU kernels run (verify_half_fu,
// at2v_verify_fu.h, compiled for the host in at2v_cpu.cpp): verdicts are identical by construction, and the oracle
// (oracle/) is never linked or called. Plain C++ declarations, so the hipcc-compiled context code can call them.
#pragma once
#include <cstddef>
#include <cstdint>

namespace at2v {

struct CpuPool;

// CPUs this process may run on: the affinity mask, capped by a cgroup v2/v1 CPU quota if one is set (a container that
// grants 16 of a host's 256 threads reports 256 in its mask).
unsigned usable_cpus();

// A pool of `threads` workers (0 = usable_cpus()); the calling thread of a batch works too, so `threads` - 1 are
// spawned. nullptr if no thread could be started.
CpuPool* cpu_pool_create(unsigned threads);
void cpu_pool_destroy(CpuPool* p);
unsigned cpu_pool_threads(const CpuPool* p);

// A pool without the verify tables, for host work of the GPU path (the staging copies of at2v_verify_batch), and its
// generic job: fn(arg, c) for c = 0..chunks-1 over the workers and the caller, synchronous. One job at a time per pool.
CpuPool* copy_pool_create(unsigned threads);
void pool_run(CpuPool* p, size_t chunks, void (*fn)(void*, size_t), void* arg);

// n records in the at2v_verify_batch layout -> ceil(n/32) verdict words (pad bits 0), synchronous. Chunks of 64 records
// own their two words, so workers never share a word. One batch at a time per pool (calls serialise).
void cpu_verify_batch(CpuPool* p, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint32_t* msg_off,
                      size_t n, int policy, uint32_t* verdicts);

// bit i of valid_words = 1 iff pts[i] decodes under dalek rules (the kernels' gu_frombytes), synchronous
void cpu_decode_points(CpuPool* p, const uint8_t* pts, size_t n, uint32_t* valid_words);

}  // namespace at2v
