// vss_build_info.cpp — the build's source stamp (include/vss.h vss_source_hash).
// VSS_SOURCE_HASH is the first 16 hex digits of sha256 over the Makefile's STAMPED list (the .hip
// sources, include/vss.h and the Makefile, in that list's order), computed at build time; the Python
// loader (vss_amd/_native.py) recomputes it from the tree and refuses a library built from other
// sources, so a stale prebuilt .so can never be the one that runs.
#include "../../include/vss.h"

#ifndef VSS_SOURCE_HASH
#error "VSS_SOURCE_HASH must be defined by the build (csrc/Makefile)"
#endif

extern "C" const char* vss_source_hash(void) { return VSS_SOURCE_HASH; }
