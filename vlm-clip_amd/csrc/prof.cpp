// Live per-kernel timing for bench.py's roofline (see include/clipmi.h clipmi_prof_*).
#include <string>
#include <vector>
#include "internal.h"

namespace {
struct Prof {
  bool armed = false;
  std::string variant;
  std::vector<hipEvent_t> ev;  // 2 per launch
  std::vector<double> flops;
  int used = 0;
  int cap = 0;
  bool filter = false;        // record only launches on `only` (which may be the null stream)
  hipStream_t only = nullptr;
} g;
}  // namespace

ProfScope::ProfScope(hipStream_t stream, const char* label, double flops) : s(stream), slot(-1) {
  if (!g.armed || g.used >= g.cap) return;
  if (label && g.variant != label) return;
  if (g.filter && stream != g.only) return;
  slot = g.used;
  (void)hipEventRecord(g.ev[2 * slot], s);
}

void ProfScope::finish(const char* label, double flops) {
  if (slot < 0) return;
  if (g.variant == label) {
    (void)hipEventRecord(g.ev[2 * slot + 1], s);
    g.flops[slot] = flops;
    g.used = slot + 1;
  }
  slot = -1;
}

extern "C" int clipmi_prof_arm(const char* variant, int max_launches) {
  CLIPMI_REQUIRE(variant && max_launches > 0, "prof_arm args");
  if ((int)g.ev.size() < 2 * max_launches) {
    for (int i = (int)g.ev.size(); i < 2 * max_launches; ++i) {
      hipEvent_t e;
      CLIPMI_HIP(hipEventCreate(&e));
      g.ev.push_back(e);
    }
  }
  g.flops.assign(max_launches, 0.0);
  g.cap = max_launches;
  g.used = 0;
  g.variant = variant;
  g.armed = true;
  return CLIPMI_OK;
}

extern "C" int clipmi_prof_stream(void* stream) {
  g.only = (hipStream_t)stream;
  g.filter = true;
  return CLIPMI_OK;
}

extern "C" int clipmi_prof_disarm(void) {
  g.armed = false;
  return CLIPMI_OK;
}

// after the stream has been synchronised: per-launch milliseconds and algorithmic FLOPs
extern "C" int clipmi_prof_read(int max, float* ms, double* flops) {
  int n = g.used < max ? g.used : max;
  for (int i = 0; i < n; ++i) {
    CLIPMI_HIP(hipEventElapsedTime(&ms[i], g.ev[2 * i], g.ev[2 * i + 1]));
    flops[i] = g.flops[i];
  }
  return n;
}
