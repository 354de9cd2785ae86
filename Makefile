# Build of the MI355X product (libldpc_hip.so + CLI front-ends) and the CPU
# oracle (test infrastructure). gfx950 only.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CSRC      = ldpcsimulation_amd/csrc
LIBDIR    = ldpcsimulation_amd/lib
BINDIR    = bin
# -ffp-contract=off: the decoder must not fuse 1+sigma*n or the quantiser
# into FMAs (bit-exact parity with the reference's plain IEEE arithmetic).
HIPFLAGS  = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -I$(CSRC) \
            -Wall -Wno-unused-result
CXXFLAGS  = -O2 -std=c++17 -ffp-contract=off -Iinclude -Wall

LIB       = $(LIBDIR)/libldpc_hip.so
OBJS      = $(LIBDIR)/obj/kernels.o $(LIBDIR)/obj/rows_fast.o $(LIBDIR)/obj/rows_pp.o $(LIBDIR)/obj/gdbf.o $(LIBDIR)/obj/bp.o $(LIBDIR)/obj/nb.o $(LIBDIR)/obj/nb_api.o $(LIBDIR)/obj/nb_graph.o $(LIBDIR)/obj/api.o $(LIBDIR)/obj/graph.o
CLIS      = $(BINDIR)/decodeMinSum $(BINDIR)/decodeNMS $(BINDIR)/decodeNormalizedMinSum $(BINDIR)/decodeOffsetMinSum \
            $(BINDIR)/decodeMNGDBF $(BINDIR)/decodeSMNGDBF $(BINDIR)/decodeATGDBF $(BINDIR)/decodeSATGDBF $(BINDIR)/decodeSMGDBF $(BINDIR)/decodeBP \
            $(BINDIR)/decodeSGDBF $(BINDIR)/decodeMGDBF $(BINDIR)/decodeStochasticNGDBF

# VFLAGS (-D switches of the A/B experiments, some of them wrong-result by design) belong
# to the *variant targets, which build into ab/ with -DLDPC_AB_BUILD; the product refuses
# them here, and the kernel sources refuse the wrong-result ones without LDPC_AB_BUILD.
PRODUCT_GOALS = all $(LIB) $(OBJS) $(CLIS)
ifneq ($(strip $(VFLAGS)),)
ifneq ($(filter $(PRODUCT_GOALS),$(if $(MAKECMDGOALS),$(MAKECMDGOALS),all)),)
$(error VFLAGS="$(VFLAGS)" is for the A/B targets (make ppvariant/fastvariant/nbvariant/...), not the product)
endif
endif

all: $(LIB) $(CLIS) oracle

$(LIBDIR)/obj:
	mkdir -p $@
$(BINDIR):
	mkdir -p $@

# -load-store-opt: keep the bit-phase LDS reads as single ds_read_b64 (2 LDS
# cycles each) instead of merged ds_read2st64_b64 (8 cycles for the same data).
KERNFLAGS = -Xclang -target-feature -Xclang -load-store-opt
# Loop headers on 32-byte boundaries: without it the ping-pong kernel's time moved
# by up to 4 % with the code layout (s_nop shifts at the kernel entry: 14.85-15.47
# ms); aligned, 14.78-14.85 ms for every shift.
ALIGNFLAGS = -falign-loops=32
# The ping-pong kernel under LLVM's max-memory-clause machine scheduler: its LDS
# reads issue in clauses ahead of their uses; 14.29-14.48 vs 14.65-14.77 ms per
# bench launch over 3 interleaved rounds, stable under code shifts;
# `make ppvariant PPSCHED= VFLAGS="-mllvm -amdgpu-sched-strategy=..."` for others.
PPSCHED ?= -mllvm -amdgpu-sched-strategy=max-memory-clause
# No SLP vectorisation where the compiler would pair scalar fp32 adds into v_pk_add_f32,
# which issues slower on gfx950 than the two plain adds it replaces (measured: EMS
# 7.85-7.95 -> 8.38-8.50 Gbit/s at 2.0 dB, fp32 layered DVB-S2 44.6 -> 42.2 ms, GDBF
# rows 21.7 -> 21.3 ms; flooding and BP equal). Explicit vector types (the fp32 row
# kernel's pairs) are not affected.
NOSLP = -fno-slp-vectorize
$(LIBDIR)/obj/kernels.o: $(CSRC)/kernels.hip $(CSRC)/kernels.h $(CSRC)/device_common.h $(CSRC)/minsum_common.h | $(LIBDIR)/obj
	$(HIPCC) $(HIPFLAGS) $(KERNFLAGS) $(NOSLP) -c -o $@ $<
$(LIBDIR)/obj/rows_fast.o: $(CSRC)/rows_fast.hip $(CSRC)/fast64.h $(CSRC)/kernels.h $(CSRC)/device_common.h $(CSRC)/minsum_common.h | $(LIBDIR)/obj
	$(HIPCC) $(HIPFLAGS) $(KERNFLAGS) -c -o $@ $<
$(LIBDIR)/obj/rows_pp.o: $(CSRC)/rows_pp.hip $(CSRC)/fast64.h $(CSRC)/kernels.h $(CSRC)/device_common.h $(CSRC)/minsum_common.h | $(LIBDIR)/obj
	$(HIPCC) $(HIPFLAGS) $(KERNFLAGS) $(ALIGNFLAGS) $(PPSCHED) -c -o $@ $<
$(LIBDIR)/obj/gdbf.o: $(CSRC)/gdbf.hip $(CSRC)/gdbf.h $(CSRC)/kernels.h $(CSRC)/device_common.h $(CSRC)/minsum_common.h | $(LIBDIR)/obj
	$(HIPCC) $(HIPFLAGS) $(NOSLP) -c -o $@ $<
$(LIBDIR)/obj/bp.o: $(CSRC)/bp.hip $(CSRC)/bp.h $(CSRC)/bp_math.h $(CSRC)/kernels.h $(CSRC)/device_common.h | $(LIBDIR)/obj
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<
$(LIBDIR)/obj/nb.o: $(CSRC)/nb.hip $(CSRC)/nb.h $(CSRC)/nb_layout.h $(CSRC)/kernels.h $(CSRC)/device_common.h | $(LIBDIR)/obj
	$(HIPCC) $(HIPFLAGS) $(NOSLP) -c -o $@ $<
$(LIBDIR)/obj/nb_api.o: $(CSRC)/nb_api.cpp $(CSRC)/nb.h $(CSRC)/nb_layout.h $(CSRC)/nb_graph.h $(CSRC)/kernels.h include/ldpc_hip.h | $(LIBDIR)/obj
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<
$(LIBDIR)/obj/nb_graph.o: $(CSRC)/nb_graph.cpp $(CSRC)/nb_graph.h $(CSRC)/nb_layout.h include/ldpc_hip.h | $(LIBDIR)/obj
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<
$(LIBDIR)/obj/api.o: $(CSRC)/api.cpp $(CSRC)/bp.h $(CSRC)/kernels.h $(CSRC)/gdbf.h $(CSRC)/graph.h include/ldpc_hip.h | $(LIBDIR)/obj
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<
$(LIBDIR)/obj/graph.o: $(CSRC)/graph.cpp $(CSRC)/graph.h | $(LIBDIR)/obj
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<
$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

# Reference-compatible CLI front-ends: the variant is fixed at compile time
# exactly as C_implementations/Makefile:58-65 does (plus decodeNMS =
# -D normalizedMS without quantisation, the BASELINE config-2 variant).
CLI_SRC = $(CSRC)/cli_minsum.cpp
CLI_LINK = -L$(LIBDIR) -lldpc_hip -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'
$(BINDIR)/decodeMinSum: $(CLI_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -o $@ $< $(CLI_LINK)
$(BINDIR)/decodeNMS: $(CLI_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -D normalizedMS -o $@ $< $(CLI_LINK)
$(BINDIR)/decodeNormalizedMinSum: $(CLI_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -D quantizeSamples -D normalizedMS -o $@ $< $(CLI_LINK)
$(BINDIR)/decodeOffsetMinSum: $(CLI_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -D quantizeSamples -D offsetMS -o $@ $< $(CLI_LINK)

$(BINDIR)/decodeBP: $(CLI_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -D beliefPropagation -o $@ $< $(CLI_LINK)

# GDBF / NGDBF front-ends: the -D switches of C_implementations/Makefile:33-53.
GDBF_SRC = $(CSRC)/cli_gdbf.cpp
$(BINDIR)/decodeMNGDBF: $(GDBF_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -D addNoise -D thresholdAdaptation -D weightSyndromes -D saturateSamples -o $@ $< $(CLI_LINK)
$(BINDIR)/decodeSMNGDBF: $(GDBF_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -D addNoise -D thresholdAdaptation -D weightSyndromes -D outputSmoothing -D saturateSamples -o $@ $< $(CLI_LINK)
$(BINDIR)/decodeATGDBF: $(GDBF_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -D thresholdAdaptation -o $@ $< $(CLI_LINK)
$(BINDIR)/decodeSATGDBF: $(GDBF_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -D thresholdAdaptation -D outputSmoothing -o $@ $< $(CLI_LINK)
$(BINDIR)/decodeSMGDBF: $(GDBF_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -D outputSmoothing -o $@ $< $(CLI_LINK)
# single-bit-flip schedules and stochastic flipping (Makefile:24-31)
$(BINDIR)/decodeSGDBF: $(GDBF_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -D sequentialmode -o $@ $< $(CLI_LINK)
$(BINDIR)/decodeMGDBF: $(GDBF_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -D modeswitching -o $@ $< $(CLI_LINK)
$(BINDIR)/decodeStochasticNGDBF: $(GDBF_SRC) $(LIB) $(CSRC)/cli_common.h | $(BINDIR)
	g++ $(CXXFLAGS) -D quantizeSamples -D quantizeProbabilities -D weightSyndromes -D saturateSamples -o $@ $< $(CLI_LINK)

# Kernel A/B variants: make variant NAME=x VFLAGS="-DLDPC_..." -> ab/libldpc_hip_x.so
variant:
	mkdir -p $(VARDIR)/obj_$(NAME)
	$(HIPCC) $(HIPFLAGS) $(KERNFLAGS) $(NOSLP) -DLDPC_AB_BUILD $(VFLAGS) -c -o $(VARDIR)/obj_$(NAME)/kernels.o $(CSRC)/kernels.hip
	$(HIPCC) $(HIPFLAGS) -DLDPC_AB_BUILD $(VFLAGS) -c -o $(VARDIR)/obj_$(NAME)/api.o $(CSRC)/api.cpp
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(VARDIR)/libldpc_hip_$(NAME).so \
	    $(VARDIR)/obj_$(NAME)/kernels.o $(VARDIR)/obj_$(NAME)/api.o $(LIBDIR)/obj/rows_fast.o $(LIBDIR)/obj/rows_pp.o $(LIBDIR)/obj/gdbf.o $(LIBDIR)/obj/bp.o $(LIBDIR)/obj/nb.o $(LIBDIR)/obj/nb_api.o $(LIBDIR)/obj/nb_graph.o $(LIBDIR)/obj/graph.o

# Fast row kernel A/B variants: make fastvariant NAME=x VFLAGS="-DLDPC_FAST_..." [FASTSRC=file] -> ab/libldpc_hip_x.so
FASTSRC ?= $(CSRC)/rows_fast.hip
fastvariant: $(OBJS)
	mkdir -p $(VARDIR)/obj_$(NAME)
	$(HIPCC) $(HIPFLAGS) $(KERNFLAGS) -DLDPC_AB_BUILD $(VFLAGS) -c -o $(VARDIR)/obj_$(NAME)/rows_fast.o $(FASTSRC)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(VARDIR)/libldpc_hip_$(NAME).so \
	    $(filter-out $(LIBDIR)/obj/rows_fast.o,$(OBJS)) $(VARDIR)/obj_$(NAME)/rows_fast.o

# Ping-pong kernel A/B variants: make ppvariant NAME=x VFLAGS="-DLDPC_PP_..." -> ab/libldpc_hip_x.so
ppvariant: $(OBJS)
	mkdir -p $(VARDIR)/obj_$(NAME)
	$(HIPCC) $(HIPFLAGS) $(KERNFLAGS) $(ALIGNFLAGS) $(PPSCHED) -DLDPC_AB_BUILD $(VFLAGS) -c -o $(VARDIR)/obj_$(NAME)/rows_pp.o $(PPSRC)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(VARDIR)/libldpc_hip_$(NAME).so \
	    $(filter-out $(LIBDIR)/obj/rows_pp.o,$(OBJS)) $(VARDIR)/obj_$(NAME)/rows_pp.o

PPSRC ?= $(CSRC)/rows_pp.hip
# A/B variant libraries (bench.py / time_code.py / bench_ems.py --lib ab/libldpc_hip_NAME.so):
# git-ignored; they ship to the GPU box only while they exist -- `make clean-ab` after an A/B session.
VARDIR ?= ab
clean-ab:
	rm -rf $(VARDIR)
# EMS kernel A/B variants: make nbvariant NAME=x VFLAGS="-DLDPC_EMS_..." [NBSRC=file] -> ab/libldpc_hip_x.so
NBSRC ?= $(CSRC)/nb.hip
nbvariant: $(OBJS)
	mkdir -p $(VARDIR)/obj_$(NAME)
	$(HIPCC) $(HIPFLAGS) $(NOSLP) -DLDPC_AB_BUILD $(VFLAGS) -c -o $(VARDIR)/obj_$(NAME)/nb.o $(NBSRC)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(VARDIR)/libldpc_hip_$(NAME).so \
	    $(filter-out $(LIBDIR)/obj/nb.o,$(OBJS)) $(VARDIR)/obj_$(NAME)/nb.o

# GDBF kernel A/B variants: make gdbfvariant NAME=x VFLAGS="-DLDPC_GDBF_..." -> ab/libldpc_hip_x.so
gdbfvariant: $(OBJS)
	mkdir -p $(VARDIR)/obj_$(NAME)
	$(HIPCC) $(HIPFLAGS) $(NOSLP) -DLDPC_AB_BUILD $(VFLAGS) -c -o $(VARDIR)/obj_$(NAME)/gdbf.o $(CSRC)/gdbf.hip
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(VARDIR)/libldpc_hip_$(NAME).so \
	    $(filter-out $(LIBDIR)/obj/gdbf.o,$(OBJS)) $(VARDIR)/obj_$(NAME)/gdbf.o

# BP kernel A/B variants: make bpvariant NAME=x VFLAGS="-DLDPC_BP_..." -> ab/libldpc_hip_x.so
bpvariant: $(OBJS)
	mkdir -p $(VARDIR)/obj_$(NAME)
	$(HIPCC) $(HIPFLAGS) -DLDPC_AB_BUILD $(VFLAGS) -c -o $(VARDIR)/obj_$(NAME)/bp.o $(CSRC)/bp.hip
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(VARDIR)/libldpc_hip_$(NAME).so \
	    $(filter-out $(LIBDIR)/obj/bp.o,$(OBJS)) $(VARDIR)/obj_$(NAME)/bp.o

# Bounds-checked device build (check.h): every schedule-derived LDS / global
# index of the kernels tested on the device, violations reported by the ABI call that
# launched them. Same sources and per-file flags as the product, plus -DLDPC_CHECK; a
# library of its own (tests/test_checked_build.py loads it in a child process).
CHKDIR    = $(LIBDIR)/checked
CHKLIB    = $(CHKDIR)/libldpc_hip_checked.so
CHK_OBJS  = $(patsubst $(LIBDIR)/obj/%.o,$(CHKDIR)/obj/%.o,$(OBJS))
CHK_HDRS  = $(wildcard $(CSRC)/*.h) include/ldpc_hip.h
FLAGS_kernels   = $(KERNFLAGS) $(NOSLP)
FLAGS_rows_fast = $(KERNFLAGS)
FLAGS_rows_pp   = $(KERNFLAGS) $(ALIGNFLAGS) $(PPSCHED)
FLAGS_gdbf      = $(NOSLP)
FLAGS_nb        = $(NOSLP)
$(CHKDIR)/obj:
	mkdir -p $@
$(CHKDIR)/obj/%.o: $(CSRC)/%.hip $(CHK_HDRS) | $(CHKDIR)/obj
	$(HIPCC) $(HIPFLAGS) $(FLAGS_$*) -DLDPC_CHECK -c -o $@ $<
$(CHKDIR)/obj/%.o: $(CSRC)/%.cpp $(CHK_HDRS) | $(CHKDIR)/obj
	$(HIPCC) $(HIPFLAGS) -DLDPC_CHECK -c -o $@ $<
$(CHKLIB): $(CHK_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(CHK_OBJS)
checked: $(CHKLIB)

oracle:
	$(MAKE) -f oracle/Makefile

ref:
	@if [ -d /root/reference/C_implementations ]; then $(MAKE) -f oracle/Makefile.ref; \
	 else echo "reference sources absent: oracle/_ref not rebuilt"; fi

clean:
	rm -rf $(LIBDIR) $(BINDIR) oracle/liboracle.so

.PHONY: all checked oracle ref clean clean-ab variant fastvariant ppvariant nbvariant gdbfvariant bpvariant

# Host-code sanitizer build: graph.cpp (the Tanner-graph compiler), nb_graph.cpp
# (the NB alist reader, GF tables, slot swizzles), cli_common.h (the CLIs' codeword files)
# and the CPU oracle under AddressSanitizer + UBSan, driven over code files.
ASAN_FLAGS = -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all
build/host_asan: tests/native/host_asan.cpp $(CSRC)/graph.cpp $(CSRC)/graph.h $(CSRC)/nb_graph.cpp $(CSRC)/nb_graph.h \
                 $(CSRC)/nb_layout.h $(CSRC)/cli_common.h oracle/ldpc_oracle.c oracle/ldpc_oracle.h
	mkdir -p build
	gcc $(ASAN_FLAGS) -std=c11 -ffp-contract=off -Ioracle -c -o build/ldpc_oracle_asan.o oracle/ldpc_oracle.c
	g++ $(ASAN_FLAGS) -std=c++17 -Iinclude -I$(CSRC) -Ioracle -o $@ tests/native/host_asan.cpp $(CSRC)/graph.cpp \
	    $(CSRC)/nb_graph.cpp build/ldpc_oracle_asan.o -lm
asan: build/host_asan
	build/host_asan $(ASAN_CODES)
.PHONY: asan
