#include <hip/hip_runtime.h>
#include <stdint.h>
typedef unsigned __int128 u128;
__device__ __forceinline__ u128 step128(u128 s, u128 a, u128 c){ return s*a + c; }
__global__ void k128(uint64_t* out, int iters, uint64_t seed){
  u128 A = ((u128)0x2360ED051FC65DA4ULL<<64) | 0x4385DF649FCCF645ULL;
  u128 s = ((u128)seed<<64) | (threadIdx.x + blockIdx.x*blockDim.x);
  u128 c = 1;
  uint64_t acc=0;
  for(int i=0;i<iters;i++){ s = step128(s, A, c); uint64_t hi=(uint64_t)(s>>64), lo=(uint64_t)s; unsigned r=hi>>58; uint64_t x=hi^lo; acc += (x>>r)|(x<<((-r)&63)); }
  out[threadIdx.x + blockIdx.x*blockDim.x]=acc;
}
