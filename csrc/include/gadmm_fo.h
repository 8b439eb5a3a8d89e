// ABI of the persistent first-order baseline engine (csrc/kernels/first_order.hip), mirrored by
// ctypes structures in gadmm_amd/ops/native.py (checked at load time by gadmm_fo_abi_layout).
#pragma once
#include "gadmm_chain.h"

enum FoAlg { FO_GD = 0, FO_DGD = 1, FO_LAG_PS = 2, FO_LAG_WK = 3, FO_IAG = 4, FO_DUALAVG = 5 };
enum FoModel { FO_LINEAR = 0, FO_LOGISTIC = 1 };

// Device-resident control block; the host zeroes it before a launch.
struct FoCtl {
  int monitored;   // last iteration the monitor has recorded
  int stop_iter;   // iteration at which the stop rule fired (0: not yet; -1: abort)
  int status;      // 1 converged (|obj - obj0| < tol), 2 iteration budget spent, 4 timeout
  int iters;       // iterations recorded
  double uploads;  // LAG: triggered uploads summed over the run
  double pad_;
};

struct FoArgs {
  int alg, model, n, d, m, max_iter, faithful, jacobi, has_tol, ring;
  unsigned epoch;
  int slots;      // upload-row slots of the table (row of iteration j in slot j % slots): 2 for the
                  // algorithms whose readers move in lock-step (every iteration reads every worker's
                  // row or flag, or the chain neighbours'), ring + 3 for IAG (one upload per iteration:
                  // a fast worker may lead a slow reader by up to `ring` + 1 iterations)
  double step;    // GD/LAG: 1/Hmax_all; DGD: step/100; IAG: step/N; dual averaging: alpha
  double lam;     // ridge inside f_n and grad f_n (logistic lambda; 0 for the linear reference)
  double obj0, tol;
  double thrd;    // LAG trigger constant
  long long timeout_ticks;
  const double* A;     // linear: (n_local, d, d) Grams of THIS rank's workers
  const double* b;     // linear: (n_local, d)
  const double* yy;    // linear: (n_local)
  const double* X;     // logistic: (n_local, m, d)
  const double* Y;     // logistic: (n_local, m) labels +-1
  const double* hsq;   // LAG-PS: Hmax_n^2 of EVERY worker (n)
  const int* sched;    // IAG: refreshing worker of iteration it at sched[it - 1]
  u32x4* tab;          // this rank's [slots][n][d] upload rows + [2][n] LAG upload flags (granules)
  u32x4* part;         // [ring][n][2] (f_n, trigger count) granules: the MONITOR rank's ring
  double* obj_trace;   // [max_iter] (monitor rank)
  double* cnt_trace;   // [max_iter] LAG uploads per iteration (monitor rank)
  long long* time_trace;  // [max_iter] s_memrealtime ticks since the monitor started (monitor rank)
  double* theta_out;   // [n_local][d]
  FoCtl* ctl;
  u32x4* xchk;         // XCD packing: as PersistArgs::xchk / xcd (gadmm_chain.h)
  int xcd, pad_x;
  // ---- several ranks (xGMI fabric; nranks == 1: one GPU, every field below at its one-GPU value).
  // This rank runs workers w_lo .. w_lo + n_local - 1 (workgroup b = worker w_lo + b); the monitor
  // workgroup (has_monitor, rank 0) follows them. Upload rows go to the tab of every rank that
  // reads them (GD / LAG / IAG: every rank replicates the server step; DGD / dual averaging: the
  // chain neighbours' ranks) with system-scope granule stores; f_n to the monitor's part ring; the
  // monitor pushes its progress and stop words (wmon, wstop) into every rank.
  int nranks, my_rank, w_lo, n_local;
  int has_monitor, pad_m;
  const int* owner;              // [n] rank of every worker (nranks > 1)
  u32x4* const* tab_push;        // [nranks] every rank's tab (own included; nranks > 1)
  int* wmon;                     // this rank's monitor-progress word (one GPU: &ctl->monitored)
  int* wstop;                    // this rank's stop word (one GPU: &ctl->stop_iter)
  int* const* wpush;             // [nranks] every rank's {wmon, wstop} pair (monitor, nranks > 1)
  double* pushc;                 // optional [n_local][2]: rows / flag granules each worker pushed to OTHER ranks
};
