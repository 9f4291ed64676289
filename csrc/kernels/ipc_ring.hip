// Stage-to-stage hand-off through a ring in the RECEIVER's HBM, mapped into the sender's process
// with HIP IPC: xGMI peer stores between the GPUs of one node (the same protocol runs between two
// processes sharing one GPU). SURVEY.md §5.8's "IPC ring with device flags", the latency-floor
// option for the reference's per-token hop (ZMQ + torch.save through a file there:
// /root/reference/utils/node_worker.py:44-67). Both sides are plain kernels on the caller's
// stream with no host synchronisation, and every index they use lives in device memory, so a
// send or a receive captured in a hipGraph is correct on every replay.
//
// Layout (bytes, all 256-B aligned):
//   inbox  (receiver memory, opened by the sender): flags[R] (u32, padded to 256 B), then R slots
//   ackbox (sender memory, opened by the receiver): acks[R] (u32)
//   state  (each endpoint's own memory):           {count, ticket, fail} - messages so far on
//                                                   this edge end, workgroups done with the current
//                                                   one, "a workgroup of this launch gave up"
// Message n of an edge uses slot n % R with epoch n / R + 1.
//
// Messages are any multiple of 4 bytes (16-B chunks + a dword tail).
// send(src, bytes): every workgroup waits until acks[slot] >= epoch - 1 (the receiver has drained
//   the slot's previous message), stores its share of src into the peer slot write-through
//   (sc0 sc1: the bytes leave this GPU's L2 for the peer's memory), drains them (vmcnt(0)) and
//   takes a ticket; the last workgroup stores flags[slot] = epoch (system scope, into the peer's
//   memory), advances count and resets the ticket.
// recv(dst, bytes): every workgroup waits until flags[slot] == epoch (system-scope loads of its own
//   memory, which the peer writes over xGMI), reads its share of the slot with sc0 sc1 loads (no
//   stale L2 / L1 copy of an earlier message can be returned), stores it into dst, drains, takes a
//   ticket; the last workgroup stores acks[slot] = epoch into the sender's memory, advances count.
// Publication and failure handling:
//  * every storing wave drains its write-through stores (vmcnt(0)) before its workgroup's ticket;
//    the ticket is an acq_rel RMW, and the last arriver publishes flags[slot] / acks[slot] with a
//    SYSTEM-scope release store, so every workgroup's payload happens-before the flag the peer
//    (another agent) reads; the consumer polls relaxed and takes ONE system-scope acquire load
//    once the value matches, then reads the slot with sc0 sc1 loads.
//  * every spin is bounded by a wall-clock budget (s_memrealtime, 100 MHz). A workgroup that
//    gives up records a code in the endpoint's sticky *err and marks the launch failed
//    (state[2]) but STILL takes its ticket, so the last arriver always completes the election,
//    resets the ticket and the failure word, and never publishes a partial message: the ring
//    state is never left half-advanced for the next launch.
//  * once *err is set (by any launch of the endpoint) every later launch is poisoned at entry: a
//    receive fills its destination with 0xFF bytes (bf16 NaN / int -1 ids) instead of reading
//    the slot, a send stores nothing, neither publishes, and the host's check() raises. A lost
//    peer therefore ends each launch within the budget and can never yield silent garbage.
#include <cstdint>
#include <cstring>

#include "common.h"

namespace {

constexpr int IPC_THREADS = 256;
constexpr int AUX_SYS = 17;  // sc0 | sc1: system-coherent (write-through / cache-bypassing) access

LSA_DEVICE unsigned ld_relaxed(const unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
LSA_DEVICE unsigned ld_acquire(const unsigned* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM); }
LSA_DEVICE void st_release(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
LSA_DEVICE unsigned ld_err(const unsigned* err) { return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

LSA_DEVICE __amdgpu_buffer_rsrc_t rsrc_n(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// thread 0: skip if the endpoint already failed, else poll *w (relaxed) until pred(value) or the
// deadline, then one acquire load; on timeout record ``code`` and mark the launch failed. The
// verdict is broadcast through LDS.
template <bool GE>
LSA_DEVICE bool wait_word(const unsigned* w, unsigned want, unsigned* err, unsigned code, long long ticks,
                          unsigned* fail, int* s_ok) {
  if (threadIdx.x == 0) {
    int ok = ld_err(err) == 0u;
    if (ok) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        const unsigned v = ld_relaxed(w);
        if (GE ? (int)(v - want) >= 0 : v == want) {
          (void)ld_acquire(w);  // orders this workgroup's slot reads after the peer's release
          break;
        }
        if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > ticks) {
          ok = 0;
          atomicMax(err, code);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    if (!ok) __hip_atomic_fetch_or(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}

// last-arriver election over the launch's workgroups (after this workgroup's memory ops
// drained); every workgroup takes a ticket, failed or not. The winner learns whether any
// workgroup of the launch failed and resets the ticket and the failure word for the next launch.
LSA_DEVICE bool last_arriver(unsigned* state, int* s_flag, int* s_failed) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const bool last =
        __hip_atomic_fetch_add(state + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    *s_flag = last;
    if (last) {
      *s_failed = __hip_atomic_exchange(state + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
      __hip_atomic_store(state + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return *s_flag != 0;
}

__global__ __launch_bounds__(IPC_THREADS) void ipc_send_kernel(const unsigned char* __restrict__ src, long long nbytes,
                                                               unsigned char* peer_slots, long long slot_bytes,
                                                               unsigned* peer_flags, const unsigned* acks, int R,
                                                               unsigned* state, unsigned* err, long long ticks) {
  __shared__ int s_ok, s_last, s_failed;
  const unsigned n = state[0];
  const int slot = (int)(n % (unsigned)R);
  const unsigned epoch = n / (unsigned)R + 1u;
  if (wait_word<true>(acks + slot, epoch - 1u, err, 1u, ticks, state + 2, &s_ok)) {
    const __amdgpu_buffer_rsrc_t dst = rsrc_n(peer_slots + (size_t)slot * slot_bytes, slot_bytes);
    const long long n16 = nbytes >> 4;
    for (long long i = (long long)blockIdx.x * IPC_THREADS + threadIdx.x; i < n16; i += (long long)gridDim.x * IPC_THREADS)
      __builtin_amdgcn_raw_buffer_store_b128(ld16(src + i * 16), dst, (int)(i * 16), 0, AUX_SYS);
    const int tail = (int)((nbytes & 15) >> 2);  // trailing dwords of a message not a multiple of 16 B
    if (blockIdx.x == 0 && (int)threadIdx.x < tail) {
      const int off = (int)(n16 * 16) + 4 * threadIdx.x;
      __builtin_amdgcn_raw_buffer_store_b32(*reinterpret_cast<const unsigned*>(src + off), dst, off, 0, AUX_SYS);
    }
  }
  if (last_arriver(state, &s_last, &s_failed) && threadIdx.x == 0 && !s_failed && ld_err(err) == 0u) {
    st_release(peer_flags + slot, epoch);
    state[0] = n + 1u;
  }
}

__global__ __launch_bounds__(IPC_THREADS) void ipc_recv_kernel(unsigned char* __restrict__ dst, long long nbytes,
                                                               const unsigned char* slots, long long slot_bytes,
                                                               const unsigned* flags, unsigned* peer_acks, int R,
                                                               unsigned* state, unsigned* err, long long ticks) {
  __shared__ int s_ok, s_last, s_failed;
  const unsigned n = state[0];
  const int slot = (int)(n % (unsigned)R);
  const unsigned epoch = n / (unsigned)R + 1u;
  const bool ok = wait_word<false>(flags + slot, epoch, err, 2u, ticks, state + 2, &s_ok);
  const __amdgpu_buffer_rsrc_t srcr = rsrc_n(slots + (size_t)slot * slot_bytes, slot_bytes);
  const u32x4_t poison = {~0u, ~0u, ~0u, ~0u};
  const long long n16 = nbytes >> 4;
  for (long long i = (long long)blockIdx.x * IPC_THREADS + threadIdx.x; i < n16; i += (long long)gridDim.x * IPC_THREADS)
    st16(dst + i * 16, ok ? __builtin_amdgcn_raw_buffer_load_b128(srcr, (int)(i * 16), 0, AUX_SYS) : poison);
  const int tail = (int)((nbytes & 15) >> 2);
  if (blockIdx.x == 0 && (int)threadIdx.x < tail) {
    const int off = (int)(n16 * 16) + 4 * threadIdx.x;
    *reinterpret_cast<unsigned*>(dst + off) = ok ? __builtin_amdgcn_raw_buffer_load_b32(srcr, off, 0, AUX_SYS) : ~0u;
  }
  if (last_arriver(state, &s_last, &s_failed) && threadIdx.x == 0 && !s_failed && ld_err(err) == 0u) {
    st_release(peer_acks + slot, epoch);
    state[0] = n + 1u;
  }
}

int grid_for(long long nbytes, int grid) {
  const long long need = ((nbytes >> 4) + IPC_THREADS - 1) / IPC_THREADS;  // >= 1 block (tail-only messages)
  long long g = grid > 0 ? grid : 32;
  if (g > need) g = need;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

// ---- host API --------------------------------------------------------------------------------
// Device buffer that another process can map: zero-filled, 256-B aligned; handle = 64 bytes.
//
// Coherence rule the ring relies on: the inbox (flags + slots) is written by the PEER GPU over
// xGMI while this GPU's receive kernel polls and reads it, and the ack box likewise. A plain
// hipMalloc buffer is coarse-grained: the HIP memory model makes a remote agent's writes to it
// visible only at kernel boundaries, because the owning GPU's L2 may keep a stale copy of a line
// that a peer has since rewritten in HBM (the sc0 sc1 bits bypass L1 and write L2 through, but do
// not make a stale local-L2 line coherent with a remote write). So these buffers are allocated
// UNCACHED (hipDeviceMallocUncached: MTYPE UC, every access goes to memory, coherent across agents
// during a kernel), falling back to fine-grained (hipDeviceMallocFinegrained: coherent across agents
// at system scope) if the uncached kind cannot be allocated or exported, and to coarse-grained only
// as a last resort. *kind reports what was used: 2 uncached, 1 fine-grained, 0 coarse (the pipeline
// refuses 0 for an edge between two GPUs: parallel/ipc_ring.py). ``first`` skips the stronger kinds
// (0 tries uncached first; 1 fine-grained first; 2 coarse only - the cost A/B of scripts/ipc_ring_check.py).
extern "C" int lsa_ipc_alloc(long long bytes, void** ptr, void* handle, int* kind, int first) {
  if (bytes <= 0 || !ptr || !handle || !kind || first < 0 || first > 2) return LSA_BAD_SHAPE;
  const unsigned flags[3] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained, hipDeviceMallocDefault};
  for (int i = first; i < 3; ++i) {
    *ptr = nullptr;
    if (hipExtMallocWithFlags(ptr, (size_t)bytes, flags[i]) != hipSuccess || !*ptr) {
      (void)hipGetLastError();
      continue;
    }
    hipIpcMemHandle_t h;
    if (hipMemset(*ptr, 0, (size_t)bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipIpcGetMemHandle(&h, *ptr) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipFree(*ptr);
      *ptr = nullptr;
      continue;
    }
    memcpy(handle, &h, sizeof(h));
    *kind = 2 - i;
    return LSA_OK;
  }
  return LSA_LAUNCH_FAILED;
}

extern "C" int lsa_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

extern "C" int lsa_ipc_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess ? LSA_OK : LSA_LAUNCH_FAILED;
}

extern "C" int lsa_ipc_close(void* ptr) { return hipIpcCloseMemHandle(ptr) == hipSuccess ? LSA_OK : LSA_LAUNCH_FAILED; }

extern "C" int lsa_ipc_free(void* ptr) { return hipFree(ptr) == hipSuccess ? LSA_OK : LSA_LAUNCH_FAILED; }

// bytes % 4 == 0, bytes <= slot_bytes, 16-B aligned src / dst; timeout_us bounds every spin
extern "C" int lsa_ipc_send(const void* src, long long bytes, void* peer_slots, long long slot_bytes, void* peer_flags,
                            const void* acks, int slots, void* state, void* err, long long timeout_us, int grid,
                            hipStream_t stream) {
  if (bytes <= 0 || bytes % 4 || bytes > slot_bytes || slot_bytes % 256 || slots < 1 || slot_bytes >= (1LL << 31))
    return LSA_BAD_SHAPE;
  if (reinterpret_cast<uintptr_t>(src) % 16) return LSA_BAD_SHAPE;
  ipc_send_kernel<<<grid_for(bytes, grid), IPC_THREADS, 0, stream>>>(
      static_cast<const unsigned char*>(src), bytes, static_cast<unsigned char*>(peer_slots), slot_bytes,
      static_cast<unsigned*>(peer_flags), static_cast<const unsigned*>(acks), slots, static_cast<unsigned*>(state),
      static_cast<unsigned*>(err), timeout_us * 100);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

extern "C" int lsa_ipc_recv(void* dst, long long bytes, const void* slots_base, long long slot_bytes, const void* flags,
                            void* peer_acks, int slots, void* state, void* err, long long timeout_us, int grid,
                            hipStream_t stream) {
  if (bytes <= 0 || bytes % 4 || bytes > slot_bytes || slot_bytes % 256 || slots < 1 || slot_bytes >= (1LL << 31))
    return LSA_BAD_SHAPE;
  if (reinterpret_cast<uintptr_t>(dst) % 16) return LSA_BAD_SHAPE;
  ipc_recv_kernel<<<grid_for(bytes, grid), IPC_THREADS, 0, stream>>>(
      static_cast<unsigned char*>(dst), bytes, static_cast<const unsigned char*>(slots_base), slot_bytes,
      static_cast<const unsigned*>(flags), static_cast<unsigned*>(peer_acks), slots, static_cast<unsigned*>(state),
      static_cast<unsigned*>(err), timeout_us * 100);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}
