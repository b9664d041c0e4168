// Compile-time A/B knobs of the engine (no experiment switch may reach a release build).
// Every AMDCRC_* knob below has its release default where it is used (engine.h, engine.cpp,
// crc_kernels.hip); overriding one is only allowed in a variant build, which also defines
// AMDCRC_VARIANT_BUILD (scripts/build_variant.sh).  The product Makefile never does, so a release
// build with any override stops here.  Variants that changed results (timing-only builds: no head
// fold, no part finishes, dropped mid-scan parts) are not in the source at all: they live as patches
// under experiments/patches/ (xp_switches.patch).  This header must be included before any default.
#pragma once

#ifndef AMDCRC_VARIANT_BUILD
#if defined(AMDCRC_W64_BLOCK) || defined(AMDCRC_XCD_CHUNK_GROUPS) || defined(AMDCRC_XCD_BLOCK) ||              \
    defined(AMDCRC_STREAM_W16) || defined(AMDCRC_SMALL_BATCH) || defined(AMDCRC_ROWS16) || defined(AMDCRC_XCD) || \
    defined(AMDCRC_XCD_MIN_CHUNKS) || defined(AMDCRC_STREAM_XCD) || defined(AMDCRC_STREAM_XCD_TILE) ||           \
    defined(AMDCRC_STREAM_XCD_MIN) || defined(AMDCRC_LANE_LIST_MAX) || defined(AMDCRC_LANE64_MAX) ||             \
    defined(AMDCRC_LIST_STREAM) || defined(AMDCRC_LIST_TWO_PER_CU) || defined(AMDCRC_LIST_STREAM64) ||            \
    defined(AMDCRC_X64_HOST_MAX) || defined(AMDCRC_R16_XCD) || defined(AMDCRC_STREAM_W8) || defined(AMDCRC_GUARD) ||     \
    defined(AMDCRC_STREAM_PRIO) || defined(AMDCRC_PRIO_ALL) || defined(AMDCRC_PRIO_EVERY) || defined(AMDCRC_PRIO_SCALE) ||   \
    defined(AMDCRC_R16_PRIO) || defined(AMDCRC_XCD_BPC) || defined(AMDCRC_XCD_WPE) || defined(AMDCRC_ES_FLAT)
#error "an AMDCRC_* A/B knob is set in a build that is not a variant build (define AMDCRC_VARIANT_BUILD: scripts/build_variant.sh)"
#endif
#endif
