# Build everything in-tree (the .so files travel to the GPU box with the snapshot).
#
#   convolutionalencdec_amd/lib/libviterbi_amd.so        HIP kernels + C ABI (include/viterbi_amd.h)
#   convolutionalencdec_amd/lib/libviterbi_legacy_k<K>.so legacy C API (include/viterbiDecoder.h,
#                                                         include/convEncode.h) for code config params/k<K>
#   oracle/...                                            test-only checker (oracle/Makefile)

HIPCC ?= /opt/rocm/bin/hipcc
CC ?= gcc
ARCH ?= gfx950
LIB := convolutionalencdec_amd/lib
CSRC := convolutionalencdec_amd/csrc

HIP_SRCS := $(CSRC)/vtb_api.hip $(CSRC)/vtb_lds_path.hip $(CSRC)/vtb_k7_lds.hip $(CSRC)/vtb_k9.hip \
            $(CSRC)/vtb_gen.hip $(CSRC)/vtb_genk.hip $(CSRC)/vtb_legacy.hip $(CSRC)/vtb_stream_gen.hip
HIP_HDRS := $(CSRC)/vtb_internal.h $(CSRC)/vtb_k7_common.h $(CSRC)/vtb_gen_trellis.h include/viterbi_amd.h
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Iinclude -I$(CSRC)

LEGACY_SRCS := $(CSRC)/legacy/convEncode.c $(CSRC)/legacy/convHelpers.c $(CSRC)/legacy/viterbiDecoder.c
LEGACY_HDRS := include/viterbiDecoder.h include/viterbiDecoderButterflyk1.h include/convEncode.h include/convHelpers.h
LEGACY_CFLAGS := -O2 -std=gnu11 -fPIC -Wall -Wno-unused-function -pthread

LEGACY_KS := 3 5 7 9 4_k2n3 3_k3n4 7n3 5n4 9n3 8n3 3s 4 6 8

.PHONY: all lib legacy oracle testprogs clean
all: lib legacy oracle testprogs

lib: $(LIB)/libviterbi_amd.so
legacy: $(foreach K,$(LEGACY_KS),$(LIB)/libviterbi_legacy_k$(K).so)

$(LIB)/obj/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(LIB)/obj
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB)/libviterbi_amd.so: $(patsubst $(CSRC)/%.hip,$(LIB)/obj/%.o,$(HIP_SRCS))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

$(LIB)/libviterbi_legacy_k%.so: $(LEGACY_SRCS) $(LEGACY_HDRS) params/k%/convCodeParams.c $(LIB)/libviterbi_amd.so
	$(CC) $(LEGACY_CFLAGS) -shared -Iparams/k$* -Iinclude -o $@ $(LEGACY_SRCS) params/k$*/convCodeParams.c \
		-L$(LIB) -lviterbi_amd -Wl,-rpath,'$$ORIGIN'

oracle: legacy
	$(MAKE) -C oracle

# C test programs run by the GPU tests (built here; the binaries travel with the tree)
TESTBIN := tests/native/build
testprogs: $(TESTBIN)/legacy_rand_mt

$(TESTBIN)/legacy_rand_mt: tests/native/legacy_rand_mt.c $(LIB)/libviterbi_legacy_k7.so $(LEGACY_HDRS)
	@mkdir -p $(TESTBIN)
	$(CC) -O2 -std=gnu11 -Wall -pthread -Iparams/k7 -Iinclude -o $@ $< params/k7/convCodeParams.c \
		-L$(LIB) -lviterbi_legacy_k7 -lviterbi_amd -Wl,-rpath,'$$ORIGIN/../../../convolutionalencdec_amd/lib'

clean:
	rm -rf $(LIB)/obj $(LIB)/*.so $(TESTBIN)
	$(MAKE) -C oracle clean
