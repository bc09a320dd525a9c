// ABI version / target query (include/aaclip.h), and the diagnostic trace buffer.
#include "common.h"

extern "C" int aaclip_abi_version(void) { return 7; }
extern "C" const char* aaclip_arch(void) { return "gfx950"; }

#ifdef AACLIP_TRACE
int trace_set_gemm(void*, void*, unsigned);
int trace_set_attention(void*, void*, unsigned);
int trace_set_rows(void*, void*, unsigned);
int trace_set_anomaly_map(void*, void*, unsigned);
#endif

extern "C" int aaclip_trace_buffer(void* records, void* counter, unsigned capacity) {
#ifdef AACLIP_TRACE
  AACLIP_REQUIRE((records && counter && capacity > 0) || (!records && !counter && capacity == 0));
  AACLIP_REQUIRE(((uintptr_t)records % 16) == 0 && ((uintptr_t)counter % 4) == 0);
  const int rc = trace_set_gemm(records, counter, capacity) | trace_set_attention(records, counter, capacity) |
                 trace_set_rows(records, counter, capacity) | trace_set_anomaly_map(records, counter, capacity);
  return rc ? AACLIP_ERR_LAUNCH : AACLIP_OK;
#else
  (void)records;
  (void)counter;
  (void)capacity;
  return AACLIP_ERR_ARG;  // not a trace build (make trace)
#endif
}
