// Error plumbing and version info for the libclipmi C ABI.
#include <cstdio>
#include <string>
#include "internal.h"

static thread_local std::string g_last_error;

void clipmi_set_error(const std::string& msg) { g_last_error = msg; }

int clipmi_fail(hipError_t e, const char* file, int line) {
  char buf[512];
  snprintf(buf, sizeof(buf), "HIP error %d (%s) at %s:%d", (int)e, hipGetErrorString(e), file, line);
  g_last_error = buf;
  return CLIPMI_ERR_HIP;
}

int clipmi_invalid(const std::string& msg) {
  g_last_error = msg;
  return CLIPMI_ERR_INVALID;
}

#ifndef CLIPMI_SRC_DIGEST
#define CLIPMI_SRC_DIGEST "unknown"
#endif

extern "C" int clipmi_version(void) { return 1; }
extern "C" const char* clipmi_build_digest(void) { return CLIPMI_SRC_DIGEST; }
extern "C" const char* clipmi_last_error(void) { return g_last_error.c_str(); }
