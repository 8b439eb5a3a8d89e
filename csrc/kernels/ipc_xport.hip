// Device-copy transport for the graph-replayed chain engine: multi-rank GADMM without RCCL.
//
// The chain engine (csrc/runtime/chain_engine.cpp) moves boundary theta rows after every phase and
// reduces the per-worker objective ring at every block end. With RCCL those are ncclSend/ncclRecv
// and ncclAllReduce. This transport does the same with two small kernels and IPC-mapped memory, so
//   * the engine's multi-rank code (plans, ghost rows, objective ring, monitor, D-GADMM re-plans)
//     runs with several processes on ONE GPU (RCCL refuses two ranks on one device), and
//   * on a node it is an RCCL-free alternative that stays inside the captured hipGraph.
//
// Every rank owns one fine-grained (uncached) mailbox, exported by IPC (parallel/ipc.py):
//   theta area  [R][n_total][d]   16-B granules; slot = code % R, code = 4 * iteration + phase
//   obj area    [2][n_total][ring] 16-B granules; parity = all-gather sequence & 1
//   coll area   [COLL_SLOTS][nranks][2 d + 8] 16-B granules: the device collectives of the large-d
//               star ADMM (reduce to the hub rank, broadcast from it, all-reduce of the objective,
//               standared_ADMM.m:66-71,86), slot = host sequence % COLL_SLOTS, row = source rank
// A send op stores its row straight into the peer's mailbox as {tag, lo, tag, hi} write-through
// granules (the data-is-flag form of chain_persistent.hip; a torn store is caught by the tags); the
// receiving rank's recv op re-reads its own mailbox row until every granule carries the expected
// tag, then writes the row into its theta table for the next phase kernel (a kernel boundary).
// Tags are salted with a per-solve epoch that lives in device memory (incremented by a kernel at
// every engine reset), so captured graphs stay valid and buffers need no re-zeroing.
// Overwrite safety: all ranks meet at every block-end all-gather, so no rank runs more than one block
// (<= ring iterations = 4 * ring codes) ahead of a reader; R = 8 * ring + 8 slots.
// Every spin has a wall-clock deadline; a stalled peer sets ctl->done = 4 on the waiting rank.
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "persist_device.h"
#include <stdlib.h>
#include <string.h>
#include <vector>

namespace {

constexpr int MAX_BATCH = 64;

struct XchgBatch {
  int n, phase, pad0, pad1;
  XchgOp op[MAX_BATCH];
};

constexpr int COLL_SLOTS = 8;

__host__ __device__ inline long coll_cmax(int d) { return 2L * d + 8; }

struct IpcXport {
  int rank, nranks, d, n_total, ring, R;
  long coll_base;           // granule index of the coll area
  u32x4* box;               // this rank's mailbox
  u32x4** d_boxes;          // device [nranks]: every rank's mailbox (own included), IPC-mapped
  unsigned* d_word;         // device [4]: [0] solve epoch, [1] all-gather sequence
  long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
  long long payload_bytes = 0, wire_bytes = 0, msgs = 0, obj_bytes = 0, coll_payload = 0, coll_wire = 0;
};

__device__ __forceinline__ void give_up(ChainCtl* ctl) {
  __hip_atomic_store(&ctl->done, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One workgroup (one wave) per op of the batch.
__global__ void __launch_bounds__(64) ipc_xchg_kernel(XchgBatch b, double* table, int d, int n_total, int R,
                                                      u32x4* const* boxes, u32x4* my_box, const unsigned* word,
                                                      ChainCtl* ctl, long long timeout_ticks) {
  // multi-rank: `done` changes only in the block-end monitor, identically on every rank, so every rank
  // skips the same exchanges
  if (ctl->done) return;
  const XchgOp o = b.op[blockIdx.x];
  const int lane = threadIdx.x;
  const unsigned code = (unsigned)(4 * ctl->iter + b.phase) & 0xfffffu;
  const unsigned tag = make_tag(word[0], (int)code);
  const long base = ((long)(code % (unsigned)R) * n_total + o.row) * d;  // granule index of the row
  const int cnt = o.count > 0 ? o.count : d;
  double* row = table + (long)o.row * d;
  if (o.is_send) {
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(boxes[o.peer] + base);
    for (int i = lane; i < cnt; i += 64) store_granule<true>(rs, i * 16, tag, row[i]);
    return;
  }
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(my_box + base);
  const unsigned long long deadline = now_ticks() + (unsigned long long)timeout_ticks;
  for (int i0 = 0; i0 < cnt; i0 += 64) {
    const int i = i0 + lane;
    double v = 0.0;
    for (int spin = 0;; ++spin) {
      const bool ok = i >= cnt || load_granule<true>(rs, i * 16, tag, &v);
      if (__all(ok)) break;
      if ((spin & 7) == 7 && now_ticks() > deadline) {
        if (lane == 0) give_up(ctl);
        return;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (i < cnt) row[i] = v;
  }
}

// Conditional row all-gather (LAG's uploads across ranks, GD_DGD_LAG.m:184-327): one workgroup per
// global worker w of the table. The rank that owns w pushes a flag granule (code phase_f, granule 0 of
// row w) to every other rank, and -- only when mask[w - w_lo] != 0 -- the row T[w] itself (code
// phase_r); every other rank polls the flag in its own mailbox and copies the row only when the flag
// says it was sent. So a worker that does not trigger moves 16 bytes per peer, not d x 16.
__global__ void __launch_bounds__(256) ipc_cond_rows_kernel(double* T, const int* mask, int n_local, int w_lo, int d,
                                                            int n_total, int R, int me, int nranks, int phase_r,
                                                            int phase_f, u32x4* const* boxes, u32x4* my_box,
                                                            const unsigned* word, ChainCtl* ctl,
                                                            long long timeout_ticks) {
  __shared__ int flag_sh;
  if (ctl->done) return;
  const int w = blockIdx.x;
  const unsigned code_r = (unsigned)(4 * ctl->iter + phase_r) & 0xfffffu;
  const unsigned code_f = (unsigned)(4 * ctl->iter + phase_f) & 0xfffffu;
  const unsigned tag_r = make_tag(word[0], (int)code_r), tag_f = make_tag(word[0], (int)code_f);
  const long base_r = ((long)(code_r % (unsigned)R) * n_total + w) * d;
  const long base_f = ((long)(code_f % (unsigned)R) * n_total + w) * d;
  double* row = T + (long)w * d;
  if (w >= w_lo && w < w_lo + n_local) {
    const int m = mask[w - w_lo];
    for (int r = 0; r < nranks; ++r) {
      if (r == me) continue;
      if (threadIdx.x == 0) store_granule<true>(rsrc_of(boxes[r] + base_f), 0, tag_f, m ? 1.0 : 0.0);
      if (m) {
        const __amdgpu_buffer_rsrc_t rs = rsrc_of(boxes[r] + base_r);
        for (int i = threadIdx.x; i < d; i += blockDim.x) store_granule<true>(rs, i * 16, tag_r, row[i]);
      }
    }
    return;
  }
  const unsigned long long deadline = now_ticks() + (unsigned long long)timeout_ticks;
  if (threadIdx.x == 0) {
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(my_box + base_f);
    double f = 0.0;
    int got = -1;
    for (int spin = 0;; ++spin) {
      if (load_granule<true>(rs, 0, tag_f, &f)) {
        got = f != 0.0 ? 1 : 0;
        break;
      }
      if ((spin & 7) == 7 && now_ticks() > deadline) break;
      __builtin_amdgcn_s_sleep(1);
    }
    flag_sh = got;
  }
  __syncthreads();
  const int got = flag_sh;
  if (got < 0) {
    if (threadIdx.x == 0) give_up(ctl);
    return;
  }
  if (!got) return;
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(my_box + base_r);
  for (int i = threadIdx.x; i < d; i += blockDim.x) {
    double v = 0.0;
    for (int spin = 0;; ++spin) {
      if (load_granule<true>(rs, i * 16, tag_r, &v)) break;
      if ((spin & 7) == 7 && now_ticks() > deadline) {
        give_up(ctl);
        return;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    row[i] = v;
  }
}

// Block-end reduction of the per-worker objective ring: every rank pushes its workers' entries into
// every rank's obj area, then reads all n_total x ring entries back into `reduced` (worker-indexed, so
// the monitor's worker-order sum is the same on every rank and equal to the single-rank sum).
__global__ void __launch_bounds__(256) ipc_allgather_kernel(const double* part, double* reduced, int ring, int n_total,
                                                            const int* lgid, int n_local, int nranks, long obj_base,
                                                            u32x4* const* boxes, u32x4* my_box, unsigned* word,
                                                            ChainCtl* ctl, long long timeout_ticks) {
  __shared__ int fail;
  if (ctl->done) return;
  if (threadIdx.x == 0) fail = 0;
  __syncthreads();
  const unsigned seq = word[1];
  const long par = seq & 1u;
  const unsigned tag = make_tag(word[0], (int)((seq + 1u) & 0xfffffu));
  for (int e = threadIdx.x; e < n_local * ring; e += blockDim.x) {
    const int li = e / ring, s = e % ring, g = lgid[li];
    const double v = part[(long)s * n_total + g];
    const long off = obj_base + (par * n_total + g) * ring + s;
    for (int r = 0; r < nranks; ++r) store_granule<true>(rsrc_of(boxes[r] + off), 0, tag, v);
  }
  const unsigned long long deadline = now_ticks() + (unsigned long long)timeout_ticks;
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(my_box + obj_base + par * n_total * ring);
  for (int e = threadIdx.x; e < n_total * ring; e += blockDim.x) {
    const int g = e / ring, s = e % ring;
    double v = 0.0;
    for (int spin = 0;; ++spin) {
      if (load_granule<true>(rs, e * 16, tag, &v)) break;
      if ((spin & 7) == 7 && now_ticks() > deadline) {
        fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    reduced[(long)s * n_total + g] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (fail) give_up(ctl);
    word[1] = seq + 1u;
  }
}

// Device collectives (one kernel per collective, thread i owns element i; order-deterministic sums):
//   kind 0 reduce:    non-root ranks push src into the root's coll row [me]; the root sums every
//                     rank's row in RANK ORDER (its own from src) into dst
//   kind 1 broadcast: the root pushes src into every other rank's row [root]; they copy it into dst
//   kind 2 allreduce: every rank pushes src into every other rank's row [me]; every rank sums all
//                     rows in rank order -> the same bits on every rank (the stop rule agrees)
// Overwrite safety: the star iteration ends in an all-reduce, so no rank is more than 3
// collectives ahead of another; COLL_SLOTS = 8. `done` (decided from the all-reduced objective, the
// same on every rank) skips the collective on every rank alike; a peer that never arrives sets
// done = 4 on the waiting rank at the deadline.
__global__ void __launch_bounds__(256) ipc_coll_kernel(int kind, int root, const double* src, double* dst, int count,
                                                       int me, int nranks, long slot_base, long cmax,
                                                       u32x4* const* boxes, u32x4* my_box, const unsigned* word,
                                                       unsigned seq, ChainCtl* ctl, long long timeout_ticks) {
  if (ctl->done) return;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const unsigned tag = make_tag(word[0], (int)(0x80000u | (seq & 0x7ffffu)));
  const double v = src[i];
  const bool pushes = kind == 2 || (kind == 0 && me != root) || (kind == 1 && me == root);
  if (pushes) {
    for (int r = 0; r < nranks; ++r) {
      if (r == me || (kind == 0 && r != root)) continue;
      store_granule<true>(rsrc_of(boxes[r] + slot_base + (long)me * cmax), i * 16, tag, v);
    }
  }
  const bool reads = kind == 2 || (kind == 0 && me == root) || (kind == 1 && me != root);
  if (!reads) return;
  const unsigned long long deadline = now_ticks() + (unsigned long long)timeout_ticks;
  double acc = 0.0;
  for (int r = 0; r < nranks; ++r) {
    if (kind == 1 && r != root) continue;
    double x = v;
    if (r != me) {
      const __amdgpu_buffer_rsrc_t rs = rsrc_of(my_box + slot_base + (long)r * cmax);
      for (int spin = 0;; ++spin) {
        if (load_granule<true>(rs, i * 16, tag, &x)) break;
        if ((spin & 7) == 7 && now_ticks() > deadline) {
          give_up(ctl);
          return;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    acc = (kind == 1) ? x : (r == 0 ? x : acc + x);
  }
  dst[i] = acc;
}

// One-way hop probe between two ranks (bench.py: ``xgmi_hop_us`` per chain boundary): one wave on each
// side ping-pongs a 64-granule row (the theta-row format of the persistent kernels, system-scope
// write-through stores into the peer's mailbox, polls of the own one) `n` times; the initiator times
// the round trips with s_memrealtime (after one untimed round that absorbs the launch skew).
// out[0] = ticks for n round trips (0: timed out), out[1] = XCC.
__global__ void __launch_bounds__(64) ipc_hop_probe_kernel(u32x4* mine, u32x4* peer, int initiator, int n,
                                                           unsigned salt, long long timeout_ticks,
                                                           unsigned long long* out) {
  const int lane = threadIdx.x;
  const __amdgpu_buffer_rsrc_t rs_peer = rsrc_of(peer), rs_mine = rsrc_of(mine);
  const unsigned long long deadline = now_ticks() + (unsigned long long)timeout_ticks;
  unsigned long long t0 = 0;
  bool good = true;
  for (int i = 1; i <= n + 1 && good; ++i) {
    if (i == 2) t0 = now_ticks();  // round 1 absorbs the two launches' skew: n timed round trips after it
    const unsigned tag = make_tag(salt, i);
    if (initiator) store_granule<true>(rs_peer, lane * 16, tag, (double)i);
    double v = 0.0;
    for (int spin = 0;; ++spin) {
      if (__all(load_granule<true>(rs_mine, lane * 16, tag, &v))) break;
      if ((spin & 63) == 63 && now_ticks() > deadline) {
        good = false;
        break;
      }
    }
    if (!initiator && good) store_granule<true>(rs_peer, lane * 16, tag, (double)i);
  }
  const unsigned long long t1 = now_ticks();
  if (lane == 0) {
    out[0] = good ? t1 - t0 : 0ull;
    out[1] = xcc_id();
  }
}

// A new epoch restarts the all-gather sequence too: a rank that returned early (ctl->done) and one
// whose all-gather timed out have advanced word[1] differently, and the parity / tag derived from
// it must agree across ranks for every later solve on this transport. The epoch salts the tags, so
// restarting the sequence at 0 cannot match a granule of an earlier epoch.
__global__ void ipc_new_epoch_kernel(unsigned* word) {
  if (threadIdx.x == 0) {
    word[0] = word[0] % 4095u + 1u;
    word[1] = 0u;
  }
}

}  // namespace

extern "C" {

long gadmm_ipc_box_bytes(int n_total, int d, int ring, int nranks) {
  const long R = 8L * ring + 8;
  return (R * n_total * d + 2L * n_total * ring + (long)COLL_SLOTS * nranks * coll_cmax(d)) * 16;
}

void* gadmm_ipc_xport_create(int rank, int nranks, int d, int n_total, int ring, void* my_box,
                             void* const* all_boxes, double timeout_s) {
  if (nranks < 1 || rank < 0 || rank >= nranks || d < 1 || n_total < 1 || ring < 1) {
    gadmm_set_error("ipc_xport_create: bad shape");
    return nullptr;
  }
  IpcXport* x = new IpcXport();
  x->rank = rank;
  x->nranks = nranks;
  x->d = d;
  x->n_total = n_total;
  x->ring = ring;
  x->R = 8 * ring + 8;
  x->coll_base = (long)x->R * n_total * d + 2L * n_total * ring;
  x->box = (u32x4*)my_box;
  x->timeout_ticks = (long long)(timeout_s * 1e8);
  if (hipMalloc((void**)&x->d_boxes, sizeof(void*) * nranks) != hipSuccess ||
      hipMalloc((void**)&x->d_word, 4 * sizeof(unsigned)) != hipSuccess) {
    gadmm_set_error("ipc_xport_create: hipMalloc failed");
    delete x;
    return nullptr;
  }
  if (hipMemcpy(x->d_boxes, all_boxes, sizeof(void*) * nranks, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(x->d_word, 0, 4 * sizeof(unsigned)) != hipSuccess) {
    gadmm_set_error("ipc_xport_create: upload failed");
    delete x;
    return nullptr;
  }
  return x;
}

int gadmm_ipc_xport_destroy(void* h) {
  IpcXport* x = (IpcXport*)h;
  if (!x) return 0;
  hipFree(x->d_boxes);
  hipFree(x->d_word);
  delete x;
  return 0;
}

// Start a new solve: every tag of the previous solve stops matching. Every rank calls it once per reset.
int gadmm_ipc_new_epoch(void* h, hipStream_t st) {
  IpcXport* x = (IpcXport*)h;
  hipLaunchKernelGGL(ipc_new_epoch_kernel, dim3(1), dim3(64), 0, st, x->d_word);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// The grouped exchange of a phase (phase: 0 after heads, 1 after tails, 2/3 eager re-plan refreshes).
int gadmm_ipc_exchange_rows(void* h, const XchgOp* ops, int nops, double* table, int d, int phase, ChainCtl* ctl,
                            hipStream_t st) {
  IpcXport* x = (IpcXport*)h;
  if (!x) {
    gadmm_set_error("ipc_exchange_rows: no transport");
    return -1;
  }
  if (d != x->d) {
    gadmm_set_error("ipc_exchange_rows: d=%d, transport built for %d", d, x->d);
    return -1;
  }
  for (int i0 = 0; i0 < nops; i0 += MAX_BATCH) {
    XchgBatch b{};
    b.n = nops - i0 < MAX_BATCH ? nops - i0 : MAX_BATCH;
    b.phase = phase;
    for (int k = 0; k < b.n; ++k) {
      b.op[k] = ops[i0 + k];
      if (b.op[k].peer < 0 || b.op[k].peer >= x->nranks || b.op[k].row < 0 || b.op[k].row >= x->n_total ||
          b.op[k].count > d) {
        gadmm_set_error("ipc_exchange_rows: bad op (peer %d, row %d)", b.op[k].peer, b.op[k].row);
        return -1;
      }
      if (b.op[k].is_send) {
        const long long c = b.op[k].count > 0 ? b.op[k].count : d;
        x->payload_bytes += c * 8;
        x->wire_bytes += c * 16;
        x->msgs += 1;
      }
    }
    hipLaunchKernelGGL(ipc_xchg_kernel, dim3(b.n), dim3(64), 0, st, b, table, d, x->n_total, x->R, x->d_boxes,
                       x->box, x->d_word, ctl, x->timeout_ticks);
  }
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// Conditional row all-gather over table T (n_total x d): see ipc_cond_rows_kernel. Codes 4 * iter +
// phase_r / phase_f (every rank issues the same calls per iteration). The bytes depend on the device
// mask, so they are not counted here: the caller derives them from its upload counts.
int gadmm_ipc_cond_rows(void* h, double* T, const int* mask, int n_local, int w_lo, int d, int phase_r, int phase_f,
                        ChainCtl* ctl, hipStream_t st) {
  IpcXport* x = (IpcXport*)h;
  if (!x || !T || !mask || !ctl || d != x->d || n_local < 0 || w_lo < 0 || w_lo + n_local > x->n_total ||
      phase_r == phase_f) {
    gadmm_set_error("ipc_cond_rows: bad arguments (d=%d transport d=%d, rows %d+%d of %d)", d, x ? x->d : -1, w_lo,
                    n_local, x ? x->n_total : -1);
    return -1;
  }
  hipLaunchKernelGGL(ipc_cond_rows_kernel, dim3(x->n_total), dim3(256), 0, st, T, mask, n_local, w_lo, d, x->n_total,
                     x->R, x->rank, x->nranks, phase_r, phase_f, x->d_boxes, x->box, x->d_word, ctl, x->timeout_ticks);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

int gadmm_ipc_allgather(void* h, const double* part, double* reduced, int ring, const int* lgid, int n_local,
                        ChainCtl* ctl, hipStream_t st) {
  IpcXport* x = (IpcXport*)h;
  if (!x || ring != x->ring) {
    gadmm_set_error("ipc_allgather: transport missing or built for another ring");
    return -1;
  }
  const long obj_base = (long)x->R * x->n_total * x->d;
  x->obj_bytes += (long long)n_local * ring * 16 * (x->nranks - 1);
  hipLaunchKernelGGL(ipc_allgather_kernel, dim3(1), dim3(256), 0, st, part, reduced, ring, x->n_total, lgid, n_local,
                     x->nranks, obj_base, x->d_boxes, x->box, x->d_word, ctl, x->timeout_ticks);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// One device collective on `st` (kind 0 reduce to root / 1 broadcast from root / 2 all-reduce, all
// sums in rank order), `seq` = the caller's collective counter (every rank calls the same sequence
// after the same gadmm_ipc_new_epoch). In place (src == dst) is allowed: a thread reads its element
// before it writes it.
int gadmm_ipc_collective(void* h, int kind, int root, const double* src, double* dst, int count, unsigned seq,
                         ChainCtl* ctl, hipStream_t st) {
  IpcXport* x = (IpcXport*)h;
  if (!x || kind < 0 || kind > 2 || root < 0 || root >= x->nranks || count < 1 || count > coll_cmax(x->d) ||
      !src || !dst || !ctl) {
    gadmm_set_error("ipc_collective: bad arguments (kind %d, root %d, count %d)", kind, root, count);
    return -1;
  }
  const long cmax = coll_cmax(x->d);
  const long slot_base = x->coll_base + (long)(seq % COLL_SLOTS) * x->nranks * cmax;
  const int R = x->nranks, me = x->rank;
  const long long sent = kind == 2 ? (long long)(R - 1) : kind == 0 ? (me != root ? 1 : 0) : (me == root ? R - 1 : 0);
  x->coll_payload += sent * count * 8;
  x->coll_wire += sent * count * 16;
  hipLaunchKernelGGL(ipc_coll_kernel, dim3((count + 255) / 256), dim3(256), 0, st, kind, root, src, dst, count, me, R,
                     slot_base, cmax, x->d_boxes, x->box, x->d_word, seq, ctl, x->timeout_ticks);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// out2: collective payload bytes this rank sent (8 B per double), collective wire bytes (16-B granules).
int gadmm_ipc_coll_counters(void* h, long long* out2) {
  IpcXport* x = (IpcXport*)h;
  out2[0] = x->coll_payload;
  out2[1] = x->coll_wire;
  return 0;
}

// Hop probe (see ipc_hop_probe_kernel): `mine` / `peer` are 64-granule rows in IPC-mapped fine-grained
// memory (the caller's own and the peer rank's), both sides launch together. Synchronous. Returns the
// median-free raw measurement: out2[0] = ticks (100 MHz) for n round trips, 0 on a timeout.
int gadmm_ipc_hop_probe(void* mine, void* peer, int initiator, int n, unsigned salt, double timeout_s,
                        unsigned long long* out2) {
  if (!mine || !peer || n < 1 || !out2) {
    gadmm_set_error("ipc_hop_probe: bad arguments");
    return -1;
  }
  unsigned long long* d_out = nullptr;
  GADMM_CHECK(hipMalloc((void**)&d_out, 2 * sizeof(unsigned long long)));
  GADMM_CHECK(hipMemset(d_out, 0, 2 * sizeof(unsigned long long)));
  hipLaunchKernelGGL(ipc_hop_probe_kernel, dim3(1), dim3(64), 0, 0, (u32x4*)mine, (u32x4*)peer, initiator, n,
                     salt & 0xfffu, (long long)(timeout_s * 1e8), d_out);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(out2, d_out, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  hipFree(d_out);
  GADMM_CHECK(e);
  return 0;
}

// out4: theta payload bytes sent, theta wire bytes (16-B granules), messages, objective-ring wire bytes.
// Counted at enqueue (a captured graph's replays are counted by the engine, see RunStats).
int gadmm_ipc_counters(void* h, long long* out4) {
  IpcXport* x = (IpcXport*)h;
  out4[0] = x->payload_bytes;
  out4[1] = x->wire_bytes;
  out4[2] = x->msgs;
  out4[3] = x->obj_bytes;
  return 0;
}

}  // extern "C"
