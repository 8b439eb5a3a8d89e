// Chain engine: the GADMM / D-GADMM / logistic-GADMM iteration loop on one MI355X rank.
//
// Per iteration (reference group_ADMM_closedForm.m:11-108 / dynamic_group_ADMM_closedForm.m:16-182):
//   head phase kernel  ->  [RCCL grouped send/recv of boundary theta]  ->  tail phase kernel
//   ->  [RCCL exchange]  ->  (every `block` iterations, multi-rank only) all-reduce of the
//   per-iteration partial-objective ring + monitor kernel.
// The sequence for `block` iterations is captured once into a hipGraph and replayed; the iteration
// counter, the stop decision and the objective trace live in device memory (ChainCtl), so a replay
// needs no host input and every kernel of an iteration past convergence returns at once. The host
// polls `done` one replay behind (async D2H into pinned memory + event), so the GPU never idles on
// the host. With several ranks every rank launches exactly the same number of replays: the stop
// decision comes from identical all-reduced values, so RCCL calls always match.
#include <hip/hip_runtime.h>
#include <string.h>
#include <vector>
#include <chrono>
#include <cstddef>
#include <thread>

#include "gadmm_common.h"
#include "gadmm_chain.h"

extern "C" {
int gadmm_chain_phase(const PhaseArgs* args, hipStream_t st);
int gadmm_chain_close(const PhaseArgs* args, hipStream_t st);
int gadmm_chain_monitor(ChainCtl* ctl, const double* reduced, int ring, int n_total, double* trace, int max_iter,
                        double obj0, double tol, hipStream_t st);
int gadmm_chain_reset(ChainCtl* ctl, int start_iter, int pending, hipStream_t st);
int gadmm_chain_dual_flush(const PhaseSlot* slots, int n_slots, int d, double rho, const double* theta, double* mu,
                           ChainCtl* ctl, hipStream_t st);
int gadmm_rccl_exchange_rows(void* h, const XchgOp* ops, int nops, double* table, int d, hipStream_t st);
int gadmm_rccl_allreduce_sum_f64(void* h, const double* send, double* recv, long count, hipStream_t st);
int gadmm_ipc_exchange_rows(void* h, const XchgOp* ops, int nops, double* table, int d, int phase, ChainCtl* ctl,
                            hipStream_t st);
int gadmm_ipc_allgather(void* h, const double* part, double* reduced, int ring, const int* lgid, int n_local,
                        ChainCtl* ctl, hipStream_t st);
int gadmm_rccl_abort(void* h);
}

struct ChainEngine {
  EngineDesc desc;
  std::vector<PhaseSlot> head, tail;
  std::vector<XchgOp> xh, xt;
  int plan_version = 0;
  hipGraphExec_t exec = nullptr;
  hipGraph_t graph = nullptr;
  int graph_block = 0, graph_plan = -1;
  ChainCtl* h_ctl = nullptr;  // pinned [2]
  hipEvent_t ev[2];
  hipEvent_t ev_sync = nullptr;
  bool graph_ok = true;
  // Watchdog of the host waits (gadmm_chain_engine_set_timeout; 0 = unbounded, the one-rank default).
  // RCCL has no deadline of its own: a graph whose send/recv never matches would block
  // hipEventSynchronize forever. With a deadline the waits poll; when it passes, an RCCL communicator
  // is aborted (its kernels observe the abort flag and exit), the stream is drained, and the run
  // returns GADMM_ENGINE_TIMEOUT -- the caller falls back with every rank (engine/multigpu.py). The IPC
  // transport's kernels have their own deadlines (done = 4) and never need the abort.
  double timeout_s = 0.0;

  int wait_event(hipEvent_t ev) {
    if (timeout_s <= 0) {
      GADMM_CHECK(hipEventSynchronize(ev));
      return 0;
    }
    const auto t0 = std::chrono::steady_clock::now();
    auto el = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
    for (int k = 0;; ++k) {
      hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) return 0;
      if (q != hipErrorNotReady) GADMM_CHECK(q);
      if (el() > timeout_s) break;
      if (k > 256) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    if (desc.comm) gadmm_rccl_abort(desc.comm);
    const auto t1 = std::chrono::steady_clock::now();
    while (hipEventQuery(ev) == hipErrorNotReady &&
           std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count() < 10.0)
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    if (hipEventQuery(ev) == hipErrorNotReady) {
      gadmm_set_error("chain engine: a host wait passed its %.3f s deadline and the stream did not drain%s",
                      timeout_s, desc.comm ? " after the RCCL abort" : "");
      return GADMM_RCCL_WEDGED;
    }
    gadmm_set_error("chain engine: a host wait passed its %.3f s deadline%s", timeout_s,
                    desc.comm ? " (RCCL communicator aborted)" : "");
    return GADMM_ENGINE_TIMEOUT;
  }

  int wait_stream() {
    GADMM_CHECK(hipEventRecord(ev_sync, desc.stream));
    return wait_event(ev_sync);
  }

  int flags_head() const {
    int f = PH_PRE_DUAL | PH_OBJ;
    return f;
  }
  int flags_tail() const {
    int f = PH_POST_DUAL | PH_OBJ | PH_FINISH;
    if (desc.nranks <= 1) f |= PH_LOCAL_STOP;
    return f;
  }

  // Row exchange of one phase through whichever data plane the engine was given. A multi-rank plan
  // without one is an error (never a null-communicator dereference).
  int exchange_ops(const std::vector<XchgOp>& ops, int phase) {
    if (ops.empty()) return 0;
    const PhaseArgs& a = desc.base;
    if (desc.xport) return gadmm_ipc_exchange_rows(desc.xport, ops.data(), (int)ops.size(), a.theta, a.d, phase,
                                                   a.ctl, desc.stream);
    if (desc.comm) return gadmm_rccl_exchange_rows(desc.comm, ops.data(), (int)ops.size(), a.theta, a.d, desc.stream);
    gadmm_set_error("chain engine: the plan has cross-rank messages but no communicator or transport");
    return -1;
  }

  int enqueue_iteration() {
    PhaseArgs a = desc.base;
    hipStream_t st = desc.stream;
    // head phase
    a.slots = desc.d_slots;
    a.n_slots = (int)head.size();
    a.flags = flags_head();
    if (a.n_slots > 0) {
      int r = gadmm_chain_phase(&a, st);
      if (r) return r;
    }
    int r = exchange_ops(xh, 0);
    if (r) return r;
    // tail phase (also closes the iteration: FINISH needs >= 1 block, see run())
    a.slots = desc.d_slots + head.size();
    a.n_slots = (int)tail.size();
    a.flags = flags_tail();
    if (a.n_slots > 0) {
      r = gadmm_chain_phase(&a, st);
      if (r) return r;
    } else {
      r = gadmm_chain_close(&a, st);
      if (r) return r;
    }
    return exchange_ops(xt, 1);
  }

  int enqueue_block(int block) {
    for (int i = 0; i < block; ++i) {
      int r = enqueue_iteration();
      if (r) return r;
    }
    if (desc.nranks > 1) {
      const PhaseArgs& a = desc.base;
      int r;
      if (desc.xport) {
        r = gadmm_ipc_allgather(desc.xport, a.part, desc.reduced, a.ring, a.lgid, a.n_local, a.ctl, desc.stream);
      } else if (desc.comm) {
        r = gadmm_rccl_allreduce_sum_f64(desc.comm, a.part, desc.reduced, (long)a.ring * a.n_total, desc.stream);
      } else {
        gadmm_set_error("chain engine: %d ranks but no communicator or transport", desc.nranks);
        r = -1;
      }
      if (r) return r;
      r = gadmm_chain_monitor(a.ctl, desc.reduced, a.ring, a.n_total, a.trace, a.max_iter, a.obj0, a.tol,
                              desc.stream);
      if (r) return r;
    }
    return 0;
  }

  void drop_graph() {
    if (exec) hipGraphExecDestroy(exec);
    if (graph) hipGraphDestroy(graph);
    exec = nullptr;
    graph = nullptr;
    graph_plan = -1;
  }

  int ensure_graph(int block) {
    if (exec && graph_block == block && graph_plan == plan_version) return 0;
    drop_graph();
    hipError_t e = hipStreamBeginCapture(desc.stream, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) {
      graph_ok = false;
      return 0;
    }
    int r = enqueue_block(block);
    hipGraph_t g = nullptr;
    e = hipStreamEndCapture(desc.stream, &g);
    if (r || e != hipSuccess || g == nullptr) {
      if (g) hipGraphDestroy(g);
      (void)hipGetLastError();
      graph_ok = false;  // fall back to eager launches (e.g. a communicator without capture support)
      return 0;
    }
    e = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
    if (e != hipSuccess) {
      hipGraphDestroy(g);
      (void)hipGetLastError();
      graph_ok = false;
      return 0;
    }
    graph = g;
    graph_block = block;
    graph_plan = plan_version;
    return 0;
  }
};

extern "C" {

void* gadmm_chain_engine_create(const EngineDesc* desc) {
  ChainEngine* e = new ChainEngine();
  e->desc = *desc;
  if (hipHostMalloc((void**)&e->h_ctl, 2 * sizeof(ChainCtl), hipHostMallocDefault) != hipSuccess) {
    gadmm_set_error("hipHostMalloc failed");
    delete e;
    return nullptr;
  }
  memset(e->h_ctl, 0, 2 * sizeof(ChainCtl));
  hipEventCreateWithFlags(&e->ev[0], hipEventDisableTiming);
  hipEventCreateWithFlags(&e->ev[1], hipEventDisableTiming);
  hipEventCreateWithFlags(&e->ev_sync, hipEventDisableTiming);
  return e;
}

void gadmm_chain_engine_destroy(void* h) {
  ChainEngine* e = (ChainEngine*)h;
  if (!e) return;
  e->drop_graph();
  hipEventDestroy(e->ev[0]);
  hipEventDestroy(e->ev[1]);
  if (e->ev_sync) hipEventDestroy(e->ev_sync);
  if (e->h_ctl) hipHostFree(e->h_ctl);
  delete e;
}

// Install a chain plan: this rank's head slots, tail slots and the p2p messages after each phase.
int gadmm_chain_engine_set_plan(void* h, int n_head, const PhaseSlot* head, int n_tail, const PhaseSlot* tail,
                                int n_xh, const XchgOp* xh, int n_xt, const XchgOp* xt) {
  ChainEngine* e = (ChainEngine*)h;
  e->head.assign(head, head + n_head);
  e->tail.assign(tail, tail + n_tail);
  e->xh.assign(xh, xh + n_xh);
  e->xt.assign(xt, xt + n_xt);
  std::vector<PhaseSlot> all(e->head);
  all.insert(all.end(), e->tail.begin(), e->tail.end());
  if (!all.empty())
    GADMM_CHECK(hipMemcpyAsync(e->desc.d_slots, all.data(), all.size() * sizeof(PhaseSlot), hipMemcpyHostToDevice,
                               e->desc.stream));
  GADMM_CHECK(hipStreamSynchronize(e->desc.stream));
  e->plan_version++;
  return 0;
}

int gadmm_chain_engine_set_scalars(void* h, double rho, double obj0, double tol, int max_iter) {
  ChainEngine* e = (ChainEngine*)h;
  const PhaseArgs& b = e->desc.base;
  // captured kernels carry these scalars by value: re-capture only when one of them changes
  if (b.rho == rho && b.obj0 == obj0 && b.tol == tol && b.max_iter == max_iter) return 0;
  e->desc.base.rho = rho;
  e->desc.base.obj0 = obj0;
  e->desc.base.tol = tol;
  e->desc.base.max_iter = max_iter;
  e->drop_graph();
  return 0;
}

// Host -> device copy queued on `st` (the D-GADMM epoch tables: one pinned staging buffer per engine,
// reused after the stream's sync; a torch copy_ per launch costs more host time than the copy itself).
int gadmm_memcpy_h2d_async(void* dst, const void* src, size_t bytes, hipStream_t st) {
  GADMM_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
  return 0;
}

extern "C" int gadmm_epoch_tables_blocked(const long long* P, int E, int n, int* slots, int* pos, int* flush);

// The blocked kernel's D-GADMM launch tables in one call (one GPU): checks the epoch starts (the first
// at start_iter, at or before it for a continuation; strictly increasing), writes [starts | slots |
// pos | flush] (gadmm_epoch_tables_blocked) straight into the pinned staging buffer `stage` and queues
// its copy to `dstage` on `st`. Replaces ~10 numpy steps per launch on the host path before the
// kernel (round 5: rp:args -> rp:tables). Returns the int32 words staged, or < 0 on an error.
long gadmm_epoch_stage_blocked(const long long* starts, const long long* P, int E, int n, int start_iter, int cont,
                               int* stage, long cap, void* dstage, hipStream_t st) {
  if (E < 1 || n < 1 || !starts || !P || !stage || !dstage) {
    gadmm_set_error("epoch_stage_blocked: bad arguments");
    return -1;
  }
  if (cont ? starts[0] > start_iter : starts[0] != start_iter) {
    gadmm_set_error("epochs must start at start_iter (continuations: at or before it)");
    return -1;
  }
  for (int e = 1; e < E; ++e)
    if (starts[e] <= starts[e - 1]) {
      gadmm_set_error("epoch starts must increase");
      return -1;
    }
  const long total = (long)E + (long)E * n * 7;  // starts, slots (4), pos (1), flush (2)
  if (total > cap) {
    gadmm_set_error("epoch_stage_blocked: staging buffer holds %ld words, %ld needed", cap, total);
    return -1;
  }
  for (int e = 0; e < E; ++e) stage[e] = (int)starts[e];
  int* slots = stage + E;
  int* pos = slots + (long)E * n * 4;
  int* flush = pos + (long)E * n;
  const int rc = gadmm_epoch_tables_blocked(P, E, n, slots, pos, flush);
  if (rc != 0) {
    gadmm_set_error("epoch tables: every chain must be a permutation (rc %d)", rc);
    return -2;
  }
  const hipError_t ce = hipMemcpyAsync(dstage, stage, (size_t)total * 4, hipMemcpyHostToDevice, st);
  if (ce != hipSuccess) {  // negative: the return value is otherwise a word count
    gadmm_set_error("epoch_stage_blocked: hipMemcpyAsync -> %s", hipGetErrorString(ce));
    return -3;
  }
  return total;
}

// Device -> host copy queued on `st` (a persistent solve's read-back block into its pinned buffer).
int gadmm_memcpy_d2h_async(void* dst, const void* src, size_t bytes, hipStream_t st) {
  GADMM_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
  return 0;
}

int gadmm_chain_engine_reset(void* h, int start_iter, int pending) {
  ChainEngine* e = (ChainEngine*)h;
  return gadmm_chain_reset(e->desc.base.ctl, start_iter, pending, e->desc.stream);
}

// Apply the pending head duals with the CURRENT plan (before a re-chain / checkpoint).
int gadmm_chain_engine_flush(void* h) {
  ChainEngine* e = (ChainEngine*)h;
  const PhaseArgs& a = e->desc.base;
  return gadmm_chain_dual_flush(e->desc.d_slots, (int)e->head.size(), a.d, a.rho, a.theta, a.mu, a.ctl,
                                e->desc.stream);
}

// Run until convergence, max_iter, or until the device iteration counter passes `stop_iter`
// (stop_iter <= 0: no limit). `block` iterations per graph replay. Returns 0 on success.
int gadmm_chain_engine_run(void* h, int block, int stop_iter, int use_graph, RunStats* out) {
  ChainEngine* e = (ChainEngine*)h;
  hipStream_t st = e->desc.stream;
  if (block < 1) block = 1;
  auto t0 = std::chrono::steady_clock::now();
  bool graph = use_graph && e->graph_ok;
  if (graph) {
    int r = e->ensure_graph(block);
    if (r) return r;
    graph = e->graph_ok && e->exec;
  }
  // Bound iterations per call so a D-GADMM epoch stops exactly at its boundary.
  int replays = 0, launched = 0;
  ChainCtl last{};
  // read the starting iteration
  GADMM_CHECK(hipMemcpyAsync(&e->h_ctl[0], e->desc.base.ctl, sizeof(ChainCtl), hipMemcpyDeviceToHost, st));
  if (int w = e->wait_stream()) return w;
  const int start = e->h_ctl[0].iter;
  if (e->h_ctl[0].done) {
    last = e->h_ctl[0];
  } else {
    int budget = stop_iter > 0 ? stop_iter - start + 1 : 0x7fffffff;
    if (budget <= 0) budget = 0;
    int k = 0;
    bool stop = false;
    while (!stop) {
      int nb = block;
      if (budget < nb) nb = budget;
      if (nb <= 0) break;
      if (graph && nb == block) {
        GADMM_CHECK(hipGraphLaunch(e->exec, st));
      } else {
        int r = e->enqueue_block(nb);
        if (r) return r;
      }
      budget -= nb;
      launched += nb;
      replays++;
      GADMM_CHECK(hipMemcpyAsync(&e->h_ctl[k & 1], e->desc.base.ctl, sizeof(ChainCtl), hipMemcpyDeviceToHost, st));
      GADMM_CHECK(hipEventRecord(e->ev[k & 1], st));
      if (k > 0) {
        if (int w = e->wait_event(e->ev[(k - 1) & 1])) return w;
        if (e->h_ctl[(k - 1) & 1].done) stop = true;  // one replay in flight beyond the decision
      }
      if (budget <= 0) stop = true;
      ++k;
    }
    if (int w = e->wait_stream()) return w;
    last = e->h_ctl[(k - 1) & 1];
  }
  auto t1 = std::chrono::steady_clock::now();
  out->wall_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  out->done = last.done;
  out->iters = last.done ? last.conv_iter : last.iter - 1;
  out->iterations_launched = launched;
  out->replays = replays;
  long long per_iter = 0, msgs = 0;
  for (auto& o : e->xh)
    if (o.is_send) { per_iter += (long long)(o.count > 0 ? o.count : e->desc.base.d) * 8; msgs++; }
  for (auto& o : e->xt)
    if (o.is_send) { per_iter += (long long)(o.count > 0 ? o.count : e->desc.base.d) * 8; msgs++; }
  const int ran = out->iters - start + 1 > 0 ? out->iters - start + 1 : 0;
  out->p2p_bytes = per_iter * ran;
  out->wire_bytes = e->desc.xport ? 2 * per_iter * ran : per_iter * ran;
  out->p2p_msgs = msgs * ran;
  // stop-rule traffic leaving this rank per block: RCCL all-reduce of the [ring][n_total] objective ring
  // (payload), or the transport's objective granules to every other rank (wire bytes, 16 B each)
  const PhaseArgs& pa = e->desc.base;
  out->monitor_bytes = e->desc.nranks <= 1 ? 0
                       : e->desc.xport ? (long long)replays * pa.n_local * pa.ring * 16 * (e->desc.nranks - 1)
                                       : (long long)replays * pa.ring * pa.n_total * 8;
  return 0;
}

int gadmm_chain_engine_set_timeout(void* h, double timeout_s) {
  ChainEngine* e = (ChainEngine*)h;
  if (!e) {
    gadmm_set_error("chain_engine_set_timeout: null engine");
    return -1;
  }
  e->timeout_s = timeout_s > 0 ? timeout_s : 0.0;
  return 0;
}

int gadmm_chain_engine_graph_ok(void* h) { return ((ChainEngine*)h)->graph_ok ? 1 : 0; }

// One eager exchange with the current plan (which = 0: after-head messages, 1: after-tail).
int gadmm_chain_engine_exchange(void* h, int which) {
  ChainEngine* e = (ChainEngine*)h;
  auto& ops = which == 0 ? e->xh : e->xt;
  if (ops.empty()) return 0;
  int r = e->exchange_ops(ops, 2 + (which != 0));  // phase codes 2/3: never collide with the in-loop 0/1
  if (r) return r;
  return e->wait_stream();
}

// ABI self-description: sizes and a few offsets of every struct shared with Python (ctypes).
int gadmm_abi_layout(long long* out, int n) {
  long long v[] = {(long long)sizeof(PhaseSlot), (long long)sizeof(XchgOp), (long long)sizeof(ChainCtl),
                   (long long)sizeof(PhaseArgs), (long long)offsetof(PhaseArgs, rho), (long long)offsetof(PhaseArgs, ring),
                   (long long)offsetof(PhaseArgs, inner_iters), (long long)sizeof(EngineDesc),
                   (long long)offsetof(EngineDesc, stream), (long long)sizeof(RunStats),
                   (long long)sizeof(PersistArgs), (long long)offsetof(PersistArgs, rho),
                   (long long)offsetof(PersistArgs, ctl), (long long)offsetof(PhaseArgs, lgid),
                   (long long)offsetof(EngineDesc, xport), (long long)offsetof(PersistArgs, xchk),
                   (long long)offsetof(PersistArgs, dl_tab), (long long)offsetof(PersistArgs, minv_pad),
                   (long long)offsetof(PersistArgs, ep_flush)};
  const int k = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < n && i < k; ++i) out[i] = v[i];
  return k;
}

}  // extern "C"
