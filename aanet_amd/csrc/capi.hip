// capi.hip -- library-level entry points of the C ABI (include/aanet_mi355x.h).
#include "common.h"

extern "C" int aanet_version(void) { return AANET_ABI_VERSION; }

extern "C" const char *aanet_status_string(int status) {
  if (status == AANET_OK) return "ok";
  if (status == AANET_EINVAL) return "invalid argument";
  if (status == AANET_EUNSUPPORTED) return "unsupported configuration";
  if (status == AANET_EABI) return "descriptor struct_size mismatch (caller built against another header version)";
  if (status > 0) return hipGetErrorString((hipError_t)status);
  return "unknown status";
}
