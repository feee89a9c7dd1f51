// Status strings / version of the libdal C ABI (include/dal.h).
#include "common.hpp"

extern "C" const char* dal_status_string(int status) {
  switch (status) {
    case DAL_OK: return "ok";
    case DAL_ERR_ARG: return "invalid argument (null pointer or bad enum)";
    case DAL_ERR_SHAPE: return "shape, padding or alignment contract violated";
    case DAL_ERR_UNSUPPORTED: return "unsupported input (e.g. tree deeper than DAL_MAX_TREE_DEPTH)";
    case DAL_ERR_HIP: return "HIP launch or attribute failure";
    case DAL_ERR_CAPACITY: return "k or candidate count above kernel capacity";
    default: return "unknown dal status";
  }
}

extern "C" int dal_abi_version(void) { return 10; }
