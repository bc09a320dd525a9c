// ABI version / target query (include/aaclip.h).
#include "common.h"

extern "C" int aaclip_abi_version(void) { return 5; }
extern "C" const char* aaclip_arch(void) { return "gfx950"; }
