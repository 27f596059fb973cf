// Live per-kernel timing for bench.py's roofline (see include/clipmi.h clipmi_prof_*).
#include <string>
#include <vector>
#include "internal.h"

namespace {
struct Prof {
  bool armed = false;
  std::vector<std::string> labels;  // the armed variant labels (comma-separated at arm time)
  std::vector<hipEvent_t> ev;       // 2 per launch
  std::vector<double> flops;
  std::vector<int> which;           // index into labels, per launch
  int used = 0;
  int cap = 0;
  bool filter = false;        // record only launches on `only` (which may be the null stream)
  hipStream_t only = nullptr;
  int find(const char* label) const {
    for (size_t i = 0; i < labels.size(); ++i)
      if (labels[i] == label) return (int)i;
    return -1;
  }
} g;
}  // namespace

ProfScope::ProfScope(hipStream_t stream, const char* label, double flops) : s(stream), slot(-1) {
  if (!g.armed || g.used >= g.cap) return;
  if (label && g.find(label) < 0) return;
  if (g.filter && stream != g.only) return;
  slot = g.used;
  (void)hipEventRecord(g.ev[2 * slot], s);
}

void ProfScope::finish(const char* label, double flops) {
  if (slot < 0) return;
  const int w = label ? g.find(label) : -1;
  if (w >= 0) {
    (void)hipEventRecord(g.ev[2 * slot + 1], s);
    g.flops[slot] = flops;
    g.which[slot] = w;
    g.used = slot + 1;
  }
  slot = -1;
}

extern "C" int clipmi_prof_arm(const char* variants, int max_launches) {
  CLIPMI_REQUIRE(variants && max_launches > 0, "prof_arm args");
  if ((int)g.ev.size() < 2 * max_launches) {
    for (int i = (int)g.ev.size(); i < 2 * max_launches; ++i) {
      hipEvent_t e;
      CLIPMI_HIP(hipEventCreate(&e));
      g.ev.push_back(e);
    }
  }
  g.labels.clear();
  std::string all(variants), cur;
  for (char c : all + ",") {
    if (c == ',') {
      if (!cur.empty()) g.labels.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  CLIPMI_REQUIRE(!g.labels.empty(), "prof_arm: no variant label");
  g.flops.assign(max_launches, 0.0);
  g.which.assign(max_launches, -1);
  g.cap = max_launches;
  g.used = 0;
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

// per launch: the index of its label in the comma-separated list given to clipmi_prof_arm
extern "C" int clipmi_prof_read_labels(int max, int* which) {
  int n = g.used < max ? g.used : max;
  for (int i = 0; i < n; ++i) which[i] = g.which[i];
  return n;
}
