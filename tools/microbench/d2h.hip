// D2H of a segment's hit slots (13 MB) into different host destinations:
// pageable, hipHostMalloc default (coherent), non-coherent, and registered
// malloc memory. Times with host wall clock around async copy + sync.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
static double Now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
  const size_t bytes = 13u << 20;
  void *dev;
  CK(hipMalloc(&dev, bytes));
  CK(hipMemset(dev, 1, bytes));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<char> pageable(bytes);
  void *pin_def, *pin_nc, *reg = malloc(bytes);
  CK(hipHostMalloc(&pin_def, bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&pin_nc, bytes, hipHostMallocNonCoherent));
  CK(hipHostRegister(reg, bytes, hipHostRegisterDefault));
  struct V { const char *name; void *p; } vs[] = {{"pageable", pageable.data()}, {"hostmalloc_default", pin_def},
                                                   {"hostmalloc_noncoherent", pin_nc}, {"registered", reg}};
  for (int rep = 0; rep < 3; ++rep)
    for (auto &v : vs) {
      const double t0 = Now();
      CK(hipMemcpyAsync(v.p, dev, bytes, hipMemcpyDeviceToHost, s));
      const double t1 = Now();
      CK(hipStreamSynchronize(s));
      const double t2 = Now();
      // host read of the result (formatting reads it)
      long sum = 0;
      for (size_t i = 0; i < bytes; i += 64) sum += ((const char *)v.p)[i];
      const double t3 = Now();
      printf("%-24s enqueue %.3f ms  copy+sync %.3f ms (%.1f GB/s)  host read %.3f ms %ld\n", v.name,
             (t1 - t0) * 1e3, (t2 - t0) * 1e3, bytes / (t2 - t0) / 1e9, (t3 - t2) * 1e3, sum);
    }
  return 0;
}
