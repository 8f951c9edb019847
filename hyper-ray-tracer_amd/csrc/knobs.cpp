/*
 * knobs.cpp — the library's A/B environment knobs, in one place.
 *
 * The reference takes its configuration as explicit arguments (src/arguments.rs:23-47).  What can change an
 * image's bits is therefore explicit here too (hrt_scene_options: BVH tie order, walk hierarchy, sample
 * chunks).  The environment variables that remain are A/B switches between bit-identical variants (kernel
 * choice, LDS staging, batch thresholds, ...).  Every read goes through knob_env, every
 * name is in KNOWN_KNOBS, and hrt_last_launch reports the set ones, so a measurement says what ran (bench.py
 * refuses a headline line with any set).
 */
#include <cstdlib>
#include <string>

#include "scene_internal.h"

namespace hrt {

const char* knob_env(const char* name) {
  const char* v = getenv(name);
  return v && *v ? v : nullptr;
}

/* every knob the library reads (tests/test_knobs.py checks this list against the sources' knob_env calls) */
static const char* const KNOWN_KNOBS[] = {
    "HRT_CLAIM_FINE",    "HRT_GEN_LDS",      "HRT_GEN_TRIM",       "HRT_GEN_WAVES_RT", "HRT_GWALK",
    "HRT_GWALK_BIG",     "HRT_GWALK_FLAT",   "HRT_GWALK_FLATLIST", "HRT_GWALK_GROUPED", "HRT_GWALK_LREF",
    "HRT_GWALK_MED", "HRT_GWALK_ONE",     "HRT_GWALK_TRIMP",  "HRT_GWALK_PACKET",  "HRT_KERNEL",         "HRT_PERLIN_LDS",   "HRT_POSTPONE",
    "HRT_PRIM_BATCH",    "HRT_SPHERE_PACKET",    "HRT_TILE_STRIDE",  "HRT_WALK_BUILD",     "HRT_WALK_DP",      "HRT_WALK_DP_SUB",
    "HRT_WALK_HOT",      "HRT_WALK_HOTSEL",  "HRT_WALK_PAYLOADS",  "HRT_WALK_SPLIT",   "HRT_WALK_C16"};

/* the knobs set in the environment now (a knob acts when read: at commit for placement knobs, at each launch
 * for the others; hrt_last_launch reports them right after a launch) */
std::string knobs_in_effect() {
  std::string out;
  for (const char* k : KNOWN_KNOBS)
    if (const char* v = knob_env(k)) {
      if (!out.empty()) out += ';';
      out += std::string(k) + "=" + v;
    }
  return out;
}

}  // namespace hrt
