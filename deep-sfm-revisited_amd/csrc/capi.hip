// Error reporting and per-kernel event profiling for libsfm_hip.
#include <mutex>
#include <vector>
#include <cstring>
#include "common.h"

namespace sfm {

static thread_local std::string g_error;

void set_error(const std::string& msg) { g_error = msg; }

Tuning& tuning() {
  static Tuning t;
  return t;
}

namespace {
struct Slot {
  std::string name;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
  double total_ms = 0.0;
  int launches = 0;
};
std::mutex g_mu;
bool g_enabled = false;
std::vector<Slot> g_slots;
std::vector<hipEvent_t> g_pool;

hipEvent_t take_event() {
  if (!g_pool.empty()) { hipEvent_t e = g_pool.back(); g_pool.pop_back(); return e; }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

int slot_of(const char* name) {
  for (size_t i = 0; i < g_slots.size(); ++i)
    if (g_slots[i].name == name) return (int)i;
  g_slots.push_back(Slot{name, {}, 0.0, 0});
  return (int)g_slots.size() - 1;
}

// Fold completed event pairs of a slot into its totals (blocks on them).
void drain(Slot& s) {
  for (auto& ev : s.events) {
    (void)hipEventSynchronize(ev.second);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ev.first, ev.second) == hipSuccess) {
      s.total_ms += ms;
      s.launches += 1;
    }
    g_pool.push_back(ev.first);
    g_pool.push_back(ev.second);
  }
  s.events.clear();
}
}  // namespace

ProfScope::ProfScope(const char* name, hipStream_t s) : slot(-1), stream(s) {
  if (!g_enabled) return;
  std::lock_guard<std::mutex> lk(g_mu);
  slot = slot_of(name);
  hipEvent_t a = take_event(), b = take_event();
  if (!a || !b) { slot = -1; return; }
  (void)hipEventRecord(a, stream);
  g_slots[slot].events.emplace_back(a, b);
}

ProfScope::~ProfScope() {
  if (slot < 0) return;
  std::lock_guard<std::mutex> lk(g_mu);
  (void)hipEventRecord(g_slots[slot].events.back().second, stream);
  if (g_slots[slot].events.size() > 256) drain(g_slots[slot]);
}

}  // namespace sfm

extern "C" {

int sfm_abi_version(void) { return SFM_ABI_VERSION; }

const char* sfm_last_error(void) { return sfm::g_error.c_str(); }

int sfm_tune_set(const char* key, int value) {
  if (!key) { sfm::set_error("sfm_tune_set: null key"); return SFM_ERR_ARG; }
  const std::string k(key);
  sfm::Tuning& t = sfm::tuning();
  if (k == "solve_lanes" && value >= 1 && value <= 64) t.solve_lanes = value;
  else if (k == "roots_lanes" && value >= 1 && value <= 64) t.roots_lanes = value;
  else if (k == "sweep_lane_pixels" && value >= 0 && value <= 2) t.sweep_lane_pixels = value;
  else if (k == "sweep_items_per_block" && (value == 1 || value == 2 || value == 4 || value == 8))
    t.sweep_items_per_block = value;
  else if (k == "sweep_flat" && value >= 0 && value <= 2) t.sweep_flat = value;
  else if (k == "sweep_nj" && (value == 1 || value == 2 || value == 4)) t.sweep_nj = value;
  else if (k == "sweep_group" && (value == 4 || value == 8)) t.sweep_group = value;
  else if (k == "score_blocks_per_cu" && value >= 1 && value <= 64) t.score_blocks_per_cu = value;
  else if (k == "score_fp32" && (value == 0 || value == 1)) t.score_fp32 = value;
  else if (k == "score_prune" && (value == 0 || value == 1)) t.score_prune = value;
  else if (k == "score_mfma" && (value == 0 || value == 1)) t.score_mfma = value;
  else if (k == "score_mf" && (value == 0 || value == 1)) t.score_mf = value;
  else if (k == "score_mf_blocks_per_cu" && value >= 1 && value <= 8) t.score_mf_blocks_per_cu = value;
  else if (k == "score_interleave" && (value == 0 || value == 1)) t.score_interleave = value;
  else if (k == "conv_rolling" && (value == 0 || value == 1)) t.conv_rolling = value;
  else if (k == "score_precision" && (value == 64 || value == 32 || value == 16)) t.score_precision = value;
  else { sfm::set_error("sfm_tune_set: unknown key or value out of range: " + k); return SFM_ERR_ARG; }
  return SFM_OK;
}

int sfm_profile_enable(int on) {
  std::lock_guard<std::mutex> lk(sfm::g_mu);
  sfm::g_enabled = on != 0;
  return SFM_OK;
}

int sfm_profile_reset(void) {
  std::lock_guard<std::mutex> lk(sfm::g_mu);
  for (auto& s : sfm::g_slots) {
    sfm::drain(s);
    s.total_ms = 0.0;
    s.launches = 0;
  }
  return SFM_OK;
}

int sfm_profile_read(const char* name, double* total_ms, int* launches) {
  if (!name || !total_ms || !launches) { sfm::set_error("sfm_profile_read: null argument"); return SFM_ERR_ARG; }
  std::lock_guard<std::mutex> lk(sfm::g_mu);
  for (auto& s : sfm::g_slots)
    if (s.name == name) {
      sfm::drain(s);
      *total_ms = s.total_ms;
      *launches = s.launches;
      return SFM_OK;
    }
  *total_ms = 0.0;
  *launches = 0;
  return SFM_OK;
}

}  // extern "C"
