/* TEST INFRASTRUCTURE ONLY.  Linked into the speedDecode harness binaries (oracle/Makefile
 * target `harness`) so that their per-second rate lines reach a redirected stdout before the
 * endless harness is stopped; the harness source itself is compiled unchanged. */
#include <stdio.h>

__attribute__((constructor)) static void linebuf_stdout(void) { setvbuf(stdout, NULL, _IOLBF, 0); }
