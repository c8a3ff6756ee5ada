// sa_registry.h — table of instantiated k_clients kernels.
#pragma once
#include "sa_internal.h"

namespace sa {
struct KernelEntry {
  int xt, ct, L, X, K;  // K: pair set (kAllPairs / kBipartite)
  LaunchFn fn;
};
#define SA_ENTRY(XT, CT, xt, ct, L, X) \
  KernelEntry { xt, ct, L, X, kAllPairs, &launch_clients<XT, CT, L, X> }
#define SA_ENTRY_K(XT, CT, xt, ct, L, X, K) \
  KernelEntry { xt, ct, L, X, K, &launch_clients<XT, CT, L, X, K> }
}  // namespace sa
