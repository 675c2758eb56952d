// Build identity of libmi355_mp.so: the hash of the native sources it was
// compiled from, passed in by the Makefile (-DMP_SOURCE_HASH, the same
// sha256 scheme as mi355_mp._lib.source_hash()).  mi355_mp._lib.load()
// refuses a library whose hash differs from the sources in the tree, so a
// stale prebuilt .so can never run (or be matched to a counter profile).
#include "../../include/mi355_mp.h"

#ifndef MP_SOURCE_HASH
#define MP_SOURCE_HASH "unknown"
#endif

extern "C" const char* mp_source_hash(void) { return MP_SOURCE_HASH; }
