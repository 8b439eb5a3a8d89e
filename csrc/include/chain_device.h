// Device-side helpers shared by the chain-engine kernels (small fused path and large-d path).
#pragma once
#include "gadmm_common.h"
#include "gadmm_chain.h"

namespace chain_dev {

__device__ __forceinline__ void drain_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ double softplus(double t) {  // log(1 + exp(t)), stable
  return t > 30.0 ? t + log1p(exp(-t)) : log1p(exp(t));
}

// Close the phase: release + ticket; the last arriver acquires and runs `finish`.
__device__ __forceinline__ bool phase_arrive(ChainCtl* ctl, int n_slots, int* flag_lds) {
  drain_vmem();
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vmem();
    const unsigned t = __hip_atomic_fetch_add(&ctl->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t == (unsigned)(n_slots - 1));
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      drain_vmem();
    }
    *flag_lds = last;
  }
  __syncthreads();
  return *flag_lds != 0;
}

__device__ __forceinline__ void finish_iteration(const PhaseArgs& a, int it) {
  if (threadIdx.x != 0) return;
  ChainCtl* ctl = a.ctl;
  if (a.tstamp && it - 1 < a.max_iter) a.tstamp[it - 1] = (long long)__builtin_amdgcn_s_memrealtime();
  if (a.flags & PH_LOCAL_STOP) {
    double s = 0.0;
    for (int i = 0; i < a.n_local; ++i) s += a.objw[i];  // fixed order (local order == worker order)
    if (it - 1 < a.max_iter) a.trace[it - 1] = s;
    const double gap = fabs(s - a.obj0);
    if (!(s == s) || isinf(s)) {
      ctl->done = 3;
      ctl->conv_iter = it;
    } else if (gap < a.tol) {
      ctl->done = 1;
      ctl->conv_iter = it;
    } else if (it >= a.max_iter) {
      ctl->done = 2;
      ctl->conv_iter = it;
    }
    ctl->monitored = it;
  } else {
    double* row = a.part + (long)((it - 1) % a.ring) * a.n_total;
    for (int i = 0; i < a.n_local; ++i) row[a.lgid[i]] = a.objw[i];
  }
  ctl->pending = 1;
  ctl->ticket = 0u;
  ctl->iter = it + 1;
}


}  // namespace chain_dev
using namespace chain_dev;
