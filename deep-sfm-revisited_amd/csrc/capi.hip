// Error reporting and per-kernel event profiling for libsfm_hip.
#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
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

static std::atomic<const char*> g_last_scorer{""};
void set_last_scorer(const char* name) { g_last_scorer.store(name, std::memory_order_relaxed); }
const char* last_scorer() { return g_last_scorer.load(std::memory_order_relaxed); }

namespace {
struct Slot {
  std::string name;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
  double total_ms = 0.0;
  int launches = 0;
};
std::mutex g_mu;
bool g_enabled = false;
std::vector<std::string> g_select;   // empty: every name is recorded
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
  if (!g_select.empty() && std::find(g_select.begin(), g_select.end(), name) == g_select.end()) return;
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

namespace {
// every tuning key: its field and accepted values
struct TuneKey {
  const char* name;
  int sfm::Tuning::*field;
  bool (*ok)(int);
};
bool v_1_64(int v) { return v >= 1 && v <= 64; }
bool v_1_16(int v) { return v >= 1 && v <= 16; }
bool v_01(int v) { return v == 0 || v == 1; }
const TuneKey kTuneKeys[] = {
    {"solve_lanes", &sfm::Tuning::solve_lanes, v_1_16},
    {"solve_coop", &sfm::Tuning::solve_coop, v_01},
    {"roots_lanes", &sfm::Tuning::roots_lanes, [](int v) { return v >= 1 && v <= 32; }},   // LDS stack columns
    {"roots_split", &sfm::Tuning::roots_split, [](int v) { return v >= 0 && v <= 2; }},
    {"sweep_lane_pixels", &sfm::Tuning::sweep_lane_pixels, [](int v) { return v >= 0 && v <= 2; }},
    {"sweep_items_per_block", &sfm::Tuning::sweep_items_per_block,
     [](int v) { return v == 1 || v == 2 || v == 4 || v == 8; }},
    {"sweep_flat", &sfm::Tuning::sweep_flat, [](int v) { return v >= 0 && v <= 3; }},
    {"sweep_buffer", &sfm::Tuning::sweep_buffer, v_01},
    {"sweep_share", &sfm::Tuning::sweep_share, v_01},
    {"sweep_store_wt", &sfm::Tuning::sweep_store_wt, [](int v) { return v >= -1 && v <= 3; }},
    {"sweep_store_nt", &sfm::Tuning::sweep_store_nt, [](int v) { return v >= 0 && v <= 2; }},
    {"sweep_store_px", &sfm::Tuning::sweep_store_px, [](int v) { return v >= -1 && v <= 8 && (v <= 2 || v == 4 || v == 8); }},
    {"sweep_run", &sfm::Tuning::sweep_run, [](int v) { return v >= 1 && v <= 1024; }},
    {"sweep_band_rows", &sfm::Tuning::sweep_band_rows, [](int v) { return v >= 2 && v <= 64; }},
    {"sweep_nj", &sfm::Tuning::sweep_nj, [](int v) { return v == 1 || v == 2 || v == 4; }},
    {"sweep_group", &sfm::Tuning::sweep_group, [](int v) { return v == 4 || v == 8; }},
    {"score_blocks_per_cu", &sfm::Tuning::score_blocks_per_cu, v_1_64},
    {"score_fp32", &sfm::Tuning::score_fp32, v_01},
    {"score_prune", &sfm::Tuning::score_prune, v_01},
    {"score_mf", &sfm::Tuning::score_mf, [](int v) { return v >= 0 && v <= 2; }},
    {"score_mf_chunk2", &sfm::Tuning::score_mf_chunk2, [](int v) { return v >= 0 && v <= 4096; }},
    {"score_mf_prune", &sfm::Tuning::score_mf_prune, [](int v) { return v == 0 || (v >= 500 && v <= 990); }},
    {"score_mf_chunk", &sfm::Tuning::score_mf_chunk, [](int v) { return v >= 1 && v <= 4096; }},
    {"score_mf_prune_margin", &sfm::Tuning::score_mf_prune_margin, [](int v) { return v >= 0 && v <= 200; }},
    {"score_mf_prune_upper", &sfm::Tuning::score_mf_prune_upper, v_01},
    {"score_mf_exact_max", &sfm::Tuning::score_mf_exact_max, [](int v) { return v >= 0 && v <= 256; }},
    {"score_mf_blocks_per_cu", &sfm::Tuning::score_mf_blocks_per_cu, [](int v) { return v >= 1 && v <= 8; }},
    {"score_interleave", &sfm::Tuning::score_interleave, v_01},
    {"conv_rolling", &sfm::Tuning::conv_rolling, v_01},
    {"score_precision", &sfm::Tuning::score_precision, [](int v) { return v == 64 || v == 32 || v == 16; }},
    {"score_lowp_template", &sfm::Tuning::score_lowp_template, v_01},
};
const TuneKey* find_key(const char* key) {
  for (const TuneKey& k : kTuneKeys)
    if (std::string(key) == k.name) return &k;
  return nullptr;
}
}  // namespace

int sfm_tune_set(const char* key, int value) {
  if (!key) { sfm::set_error("sfm_tune_set: null key"); return SFM_ERR_ARG; }
  const TuneKey* k = find_key(key);
  if (!k || !k->ok(value)) {
    sfm::set_error("sfm_tune_set: unknown key or value out of range: " + std::string(key));
    return SFM_ERR_ARG;
  }
  sfm::tuning().*(k->field) = value;
  return SFM_OK;
}

int sfm_tune_get(const char* key, int* value) {
  if (!key || !value) { sfm::set_error("sfm_tune_get: null argument"); return SFM_ERR_ARG; }
  const TuneKey* k = find_key(key);
  if (!k) { sfm::set_error("sfm_tune_get: unknown key: " + std::string(key)); return SFM_ERR_ARG; }
  *value = sfm::tuning().*(k->field);
  return SFM_OK;
}

const char* sfm_tune_key(int index) {
  const int n = (int)(sizeof(kTuneKeys) / sizeof(kTuneKeys[0]));
  return (index >= 0 && index < n) ? kTuneKeys[index].name : nullptr;
}

const char* sfm_last_scorer(void) { return sfm::last_scorer(); }

int sfm_profile_enable(int on) {
  std::lock_guard<std::mutex> lk(sfm::g_mu);
  sfm::g_enabled = on != 0;
  return SFM_OK;
}

int sfm_profile_select(const char* names) {
  std::lock_guard<std::mutex> lk(sfm::g_mu);
  sfm::g_select.clear();
  if (!names) return SFM_OK;
  std::string cur;
  for (const char* c = names;; ++c) {
    if (*c == ',' || *c == '\0') {
      if (!cur.empty()) sfm::g_select.push_back(cur);
      cur.clear();
      if (*c == '\0') break;
    } else {
      cur += *c;
    }
  }
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
