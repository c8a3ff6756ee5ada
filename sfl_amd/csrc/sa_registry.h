// sa_registry.h — table of instantiated k_clients kernels.
#pragma once
#include "sa_internal.h"

namespace sa {
struct KernelEntry {
  int xt, ct, L, X;
  LaunchFn fn;
};
#define SA_ENTRY(XT, CT, xt, ct, L, X) \
  KernelEntry { xt, ct, L, X, &launch_clients<XT, CT, L, X> }
}  // namespace sa
