// error sink for the standalone GEMM probe library (tools/dbg/gemm_mfma_probe.py)
#include <cstdarg>
#include <cstdio>
namespace mp {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
}
}  // namespace mp
