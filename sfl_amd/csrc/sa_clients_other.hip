// sa_clients_other.hip — single-client masking kernels for the non-fp32
// arithmetic types numpy promotion can produce in the reference's
// `datum * weight` (float64 data or weights, int64 data): up to 8 streams
// per pass, i.e. up to 9 parties per pass (more parties take several passes).
#include "sa_clients_impl.h"
#include "sa_registry.h"

namespace sa {

#define E(XT, CT, xt, ct)                                                                   \
  SA_ENTRY(XT, CT, xt, ct, 1, 0), SA_ENTRY(XT, CT, xt, ct, 1, 1),                           \
      SA_ENTRY(XT, CT, xt, ct, 1, 2), SA_ENTRY(XT, CT, xt, ct, 1, 3),                       \
      SA_ENTRY(XT, CT, xt, ct, 1, 4), SA_ENTRY(XT, CT, xt, ct, 1, 5),                       \
      SA_ENTRY(XT, CT, xt, ct, 1, 6), SA_ENTRY(XT, CT, xt, ct, 1, 7),                       \
      SA_ENTRY(XT, CT, xt, ct, 1, 8)

// host-only table (a function-local static, so the device pass instantiates
// the kernels without emitting host function pointers)
LaunchFn find_other_kernel(int xt, int ct, int L, int X) {
  static const KernelEntry table[] = {
      E(float, double, SA_F32, SA_F64),
      E(double, double, SA_F64, SA_F64),
      E(long long, long long, SA_I64, SA_I64),
      E(long long, double, SA_I64, SA_F64),
  };
  for (const KernelEntry& e : table)
    if (e.xt == xt && e.ct == ct && e.L == L && e.X == X) return e.fn;
  return nullptr;
}
#undef E

}  // namespace sa
