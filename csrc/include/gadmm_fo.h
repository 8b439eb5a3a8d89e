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
  int pad_;
  double step;    // GD/LAG: 1/Hmax_all; DGD: step/100; IAG: step/N; dual averaging: alpha
  double lam;     // ridge inside f_n and grad f_n (logistic lambda; 0 for the linear reference)
  double obj0, tol;
  double thrd;    // LAG trigger constant
  long long timeout_ticks;
  const double* A;     // linear: (n, d, d) Grams
  const double* b;     // linear: (n, d)
  const double* yy;    // linear: (n)
  const double* X;     // logistic: (n, m, d)
  const double* Y;     // logistic: (n, m) labels +-1
  const double* hsq;   // LAG-PS: Hmax_n^2
  const int* sched;    // IAG: refreshing worker of iteration it at sched[it - 1]
  u32x4* tab;          // [2][n][d] gradient / dual-variable granules
  u32x4* part;         // [ring][n][2] (f_n, trigger count) granules
  double* obj_trace;   // [max_iter]
  double* cnt_trace;   // [max_iter] LAG uploads per iteration
  long long* time_trace;  // [max_iter] s_memrealtime ticks since the monitor started
  double* theta_out;   // [n][d]
  FoCtl* ctl;
  u32x4* xchk;         // XCD packing: as PersistArgs::xchk / xcd (gadmm_chain.h)
  int xcd, pad_x;
};
