// Shared host/device layout of the chain engine (GADMM / D-GADMM / logistic GADMM).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Device-resident control block of one solve. Everything the iteration kernels need to decide
// "what iteration is this / are we done" lives here, so captured hipGraphs replay without host
// involvement and the host only polls `done`.
struct ChainCtl {
  int iter;        // next iteration to run (1-based, reference numbering)
  int done;        // 0 running, 1 converged (gap < tol), 2 hit max_iter, 3 numerical failure
  int conv_iter;   // first iteration whose gap < tol (reference `Iter`)
  int pending;     // heads' end-of-iteration dual update still to apply (lazy dual, see phase kernel)
  unsigned ticket; // arrival counter of the current phase kernel
  int monitored;   // last iteration whose global objective has been checked
  int placed;      // persistent kernels' XCD placement (PersistArgs::xcd): 0 not packed, 1 packed
                  // (blocks b % 8 dealt) but not verified on one XCD (system-scope stores), 2 verified
  int inner_fail;  // local Newton solves that stopped at the step cap without converging (sticky; reset
                   // zeroes it): the host re-solves with exact Newton (no chord steps) when it is set
};

// One slot of a phase plan: the local worker that updates in this phase and its chain neighbours.
struct PhaseSlot {
  int li;     // local worker index (row of the per-worker device arrays)
  int gid;    // global worker id (row of the theta table)
  int left;   // global id of the left chain neighbour, -1 at the chain head
  int right;  // global id of the right chain neighbour, -1 at the chain tail
};

enum PhaseFlags : int {
  PH_PRE_DUAL = 1,   // apply the pending (lazy) dual update of this slot's worker first (static chain heads)
  PH_POST_DUAL = 2,  // apply this slot's dual update after the solve (tails: both neighbours are fresh)
  PH_OBJ = 4,        // write the worker's local objective f_n(theta_n)
  PH_FINISH = 8,     // last arriving block closes the iteration (objective sum / stop / iter++)
  PH_LOCAL_STOP = 16 // this rank owns every worker: decide convergence on the spot
};

enum ModelKind : int { MODEL_LINEAR = 0, MODEL_LOGISTIC = 1 };

// One point-to-point message of the chain exchange: a row of the theta table to/from a peer rank.
struct XchgOp {
  int peer;     // rank
  int row;      // row of the theta table (global worker id)
  int is_send;  // 1 send, 0 recv
  int count;    // doubles (0 -> d)
};

// Arguments of one phase launch (passed by value; every pointer is a device address).
struct PhaseArgs {
  int d, n_slots, n_local, nvar;
  int deg_to_var[3];
  int flags, model;
  const PhaseSlot* slots;
  const double* Minv;  // [n_local][nvar][d][d]
  const double* A;     // [n_local][d][d]
  const double* b;     // [n_local][d]
  const double* yy;    // [n_local]
  double* mu;          // [n_local][d]
  double* theta;       // [n_total][d]
  double rho;
  double* objw;        // [n_local]
  ChainCtl* ctl;
  double* trace;       // [max_iter]
  double* part;        // [ring][n_total] per-worker objectives (multi-rank; gid-indexed, others stay 0)
  int ring, max_iter;
  double obj0, tol;
  // logistic
  const double* X;     // [n_local][m][d]
  const double* Y;     // [n_local][m]
  int m, max_inner;
  double lam, step, inner_tol;
  int* inner_iters;    // [n_local] diagnostics: inner GD steps used in the last update
  // large-d (d > 256) row-blocked path
  double* rbuf;        // [n_local][d] right-hand sides of the current phase
  int obj_mode;        // 0: exact (second GEMV with A), 1: A th = r - deg rho th (no second matrix pass)
  int solver;          // logistic local solve: 0 inexact inner GD (logReg_GD.m), 1 exact Newton (chain_newton.hip)
  // multi-rank stop rule: every rank files its workers' f_n into part[slot][gid]; the monitor sums
  // all n_total entries in worker order, the order of the single-rank finish, so the objective trace
  // is bit-identical for any rank count
  int n_total, pad_nt;
  const int* lgid;     // [n_local] global worker id of each local row
  long long* tstamp;   // optional [max_iter] s_memrealtime (100 MHz) when each iteration was decided
  // optional K4 primal residual: every tail writes ||th_l - th||^2 + ||th - th_r||^2 of iteration it
  // (its two chain edges; each edge has exactly one tail end) into rres[(it - 1) * n_total + gid]
  double* rres;        // [max_iter][n_total] or null
};

// Engine construction arguments (Python mirrors it in gadmm_amd/ops/native.py).
struct EngineDesc {
  PhaseArgs base;          // pointers, model params; slots / n_slots / flags filled per phase
  PhaseSlot* d_slots;      // device buffer, capacity >= 2 * n_local (head plan then tail plan)
  double* reduced;         // device [ring][n_total] (multi-rank)
  void* comm;              // RcclComm* or null (single rank)
  hipStream_t stream;
  int nranks;
  void* xport;             // IpcXport* (device-copy transport, csrc/kernels/ipc_xport.hip) or null: when set
                           // it replaces RCCL for the row exchange and the stop-rule reduction
};

struct RunStats {
  int iters;               // reference `Iter` (first iteration with gap < tol, or last run)
  int done;                // ChainCtl::done
  int iterations_launched; // iterations enqueued (>= iters; the rest returned early)
  int replays;
  double wall_ms;
  long long p2p_bytes;     // bytes this rank sent over the chain, iterations 1..iters
  long long p2p_msgs;
  long long monitor_bytes; // stop-rule traffic leaving this rank (see gadmm_chain_engine_run)
  long long wire_bytes;    // p2p bytes on the wire: 16-B granules per double with the IPC transport,
                           // = p2p_bytes with RCCL (its protocol framing is not visible here)
};


// Persistent single-launch solve (csrc/kernels/chain_persistent.hip). One workgroup per local worker
// (+ the stop-rule monitor on the monitor rank). Multi-GPU ("xgmi" fabric): every granule buffer is
// fine-grained device memory shared by IPC; boundary theta is pushed into the neighbour GPU's table,
// objective granules into the monitor's ring, decisions into every rank's ring.
struct PersistArgs {
  int d, n, n_local, start_iter, max_iter, lag, ring, nvar, obj_mode;
  int deg_to_var[3];
  int pending_in, has_monitor, nranks, sys_scope;
  unsigned epoch;           // salts every tag: tag = epoch << 20 | iteration (no re-zeroing between solves)
  int blk_pw;               // temporal blocking: chain positions per wave (1: 12-wave kernel, 2: paired 8-wave)
  double rho, obj0, tol;
  long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
  const PhaseSlot* slots;   // [n_local] (li, gid, left, right) in launch order
  const int* pos;           // [n_local] chain position of each slot (even = head)
  const double* Minv;       // [n_local][nvar][d][d]
  const double* A;          // [n_local][d][d]   (obj_mode 0)
  const double* b;          // [n_local][d]
  const double* yy;         // [n_local]
  double* theta;            // [n][d]   in: initial (local + ghost rows), out: final local rows
  double* mu;               // [n_local][d]   in/out
  u32x4* thg;               // [n][d]   this rank's theta granule table
  u32x4* const* push;       // [n_local * 2] remote theta tables this worker also publishes into
  u32x4* objg;              // [ring][n] the monitor rank's objective ring (remote unless monitor rank)
  unsigned long long* decg; // [ring]  this rank's decision ring
  unsigned long long* const* dec_push;  // [nranks] every rank's decision ring (monitor only)
  double* trace;            // [max_iter] (monitor rank)
  ChainCtl* ctl;
  long long* timeline;      // optional [n_local + 1][timeline_iters][8] s_memrealtime stamps (debug profiling)
  int timeline_iters;
  int blk_k;                // temporal blocking: iterations between halo exchanges (0: auto, -1: off)
  int blk_len;              // temporal blocking: chain positions owned per workgroup (0: auto)
  int n_epochs;             // D-GADMM in one launch: > 0 = number of chain epochs in this launch
  u32x4* blk_tab;           // [2][n][2][d] (theta, mu) granules of the halo exchange
  const int* epoch_start;   // [n_epochs] first iteration of each epoch (epoch_start[0] == start_iter)
  const PhaseSlot* ep_slots;  // [n_epochs][n_local] slot of local worker b (li == b) in each epoch
  const int* ep_pos;        // [n_epochs][n_local] chain position of local worker b in each epoch
  // temporal blocking across GPUs (xGMI): this rank owns chain positions [seg_lo, seg_hi]; its
  // workgroups compute [seg_lo - 2k, seg_hi + 2k]; owned (theta, mu) are also pushed into the
  // exchange tables of the peers whose computed range [peer_lo, peer_hi] contains them.
  int seg_lo, seg_hi;       // seg_hi < 0: the whole chain (one GPU)
  int blk_npeer, dbg;       // dbg: experiment bits (0 in production; see chain_blocked.hip)
  int blk_peer_lo[8], blk_peer_hi[8];
  u32x4* const* blk_peer_tab;  // [blk_npeer] peers' exchange tables (IPC-mapped)
  // real clock: the monitor stamps s_memrealtime (100 MHz) when it decides each iteration
  long long* tstamp;        // optional [max_iter]
  // D-GADMM across GPUs (per-worker kernel): theta^j of local worker b goes to every rank in
  // ep_push[epoch(j)][b], plus ep_push[epoch(j)+1][b] when j + 1 starts the next epoch (its new
  // neighbours read theta^j as their previous-iteration value); peer_thg[r] is rank r's table
  const unsigned* ep_push;  // [n_epochs][n_local] rank bitmask (own rank excluded)
  u32x4* const* peer_thg;   // [nranks]
  double* rres;             // optional K4 primal residual [max_iter][n] (see PhaseArgs::rres; owned tails)
  // D-GADMM epoch chunks (per-worker kernel): no iteration beyond hard_stop runs (> 0); the monitor
  // then reports done = 5 unless it decided a stop first. cont = 1: this launch continues a chunked
  // solve with the SAME tag salt, so the tables still hold theta^{start_iter - 1} (heads wait for it,
  // and a head's pending dual is flushed with epoch 0's -- the previous chunk's last -- chain).
  int hard_stop, cont;
  // XCD packing (one GPU, speed only): xcd = 1 launches an 8x wider grid whose blocks b % 8 != 0
  // exit at once, dealing every working block onto one XCD; xcd = 2 also has the blocks post their
  // XCC_ID into xchk ([XCHK] granules) and, if all agree, publish granules
  // with plain stores that stay in that XCD's L2 (MI355X_MICROARCH.md price list). The env
  // GADMM_XCD overrides xcd (A/B runs). xtag: the granules' tag, fresh per launch (set by the
  // launcher, gadmm_next_xtag), so xchk needs no memset in front of the kernel (a 4.8 us fill on the
  // GPU timeline of every solve, profiles/r06_dgadmm).
  u32x4* xchk;
  int xcd, xtag;
  // Data-local temporal blocking across GPUs (chain_blocked_kernel, blk_dl = 1; engine/blocked_xgmi.py
  // data_local=True): the workgroups of a rank compute ONLY its own segment [seg_lo, seg_hi] (no other
  // rank's shards), blocked inside it as on one GPU; a position at a rank boundary exchanges theta with
  // the neighbouring rank's boundary position EVERY phase through the theta ring of blk_tab: the owner
  // pushes theta^j of position p into the neighbour rank's ring (slot j % ring, row p, tag j), readers
  // poll their own ring (group_ADMM_closedForm.m:18-27,62-70: only theta crosses, never mu).
  // dl_tab[0] / [1]: blk_tab of the rank owning seg_lo - 1 / seg_hi + 1 (null at the chain ends).
  // dl_halo = 1: the boundary tail's wave also solves the other rank's boundary head from that head's
  // shard (Minv / b / mu rows of the ext range, slots[h].li), one hop per iteration on the critical
  // cycle instead of two (chain_blocked.hip; one workgroup per segment, every segment >= 2 positions).
  int blk_dl, dl_halo;
  u32x4* dl_tab[2];
  // D-GADMM in the blocked kernel (DYN): the cached inverses as lane-major images of the quad register
  // layout, zero beyond d ([n_local][nvar][gadmm_chain_blocked_pad_len(d)], engine/chain_engine.py:
  // quad_pad_image), so a re-chain reloads a position's inverse with coalesced unmasked 16-byte loads:
  // the bounds masks of a d x d reload are loop-invariant, and hoisted out of the main loop they held
  // ~100 SGPRs for the whole solve (spilled into VGPR lanes, which spilled the inverse itself to
  // scratch in every GEMV). Null outside DYN.
  const double* minv_pad;
  // DYN: per (epoch, chain position) the OLD chain neighbours (worker ids, -1: none) of the worker
  // the epoch puts there, when that worker was a head of the old chain (its pending dual is flushed
  // with them at the re-chain), as int pairs [n_epochs][n][2]. Built on the host, so a re-chain
  // issues two independent table loads instead of a chain of three dependent ones.
  const int* ep_flush;
};
constexpr int XCHK = 256;  // placement-check granules (>= workgroups of any XCD-packed launch)
