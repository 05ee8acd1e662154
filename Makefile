# Top-level build: the MI355X scorer library (HIP kernels + C-ABI + C++ host-side scorer
# classes), the C++ protocol test driver, and the (test-only) oracle.  No cmake; hipcc for gfx950.
ROCM_PATH ?= /opt/rocm
HIPCC    ?= $(ROCM_PATH)/bin/hipcc
ARCH     ?= gfx950
BUILD     = build
LIBDIR    = rasr_amd/lib
HIPFLAGS  = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result
# quantized kernels: MFMA results straight into VGPRs (gfx950 has one unified register file),
# so the v_lshl_add / v_min3 epilogue reads them without v_accvgpr_read copies.
I8FLAGS   = -mllvm -amdgpu-mfma-vgpr-form
# float kernels: default AGPR accumulators (measured faster for the f32 MFMA chains), see DESIGN.md "Measurements"
F32FLAGS  =
# split-f16 float kernel; no SLP packing: the diagonal-sum epilogue's adds were packed into v_pk_add_f32 /
# v_pk_mul_f32, which issue slower than two scalar ops beside the MFMAs (A/B: -1.0 %; no packed ops elsewhere)
SPLITFLAGS = -mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize
HOSTFLAGS = -O2 -std=c++17 -fPIC -ffp-contract=off -Wall

SRC       = rasr_amd/csrc
HDRS      = include/rasr_gmm.h $(SRC)/gmm_presel.hh $(SRC)/gmm_prepare.hh $(SRC)/gmm_kernels.hh $(SRC)/gmm_device.hh \
            $(SRC)/host/GpuFeatureScorer.hh $(SRC)/gmm_hostio.hh include/rasr_gmm_io.h include/rasr_nn.h $(SRC)/nn_kernels.hh $(SRC)/gmm_shard.hh

LIB       = $(LIBDIR)/librasr_gmm.so
OBJS      = $(BUILD)/gmm_kernels_i8.o $(BUILD)/gmm_kernels_f32.o $(BUILD)/gmm_kernels_split.o $(BUILD)/gmm_api.o $(BUILD)/gmm_prepare.o \
            $(BUILD)/GpuFeatureScorer.o $(BUILD)/MixtureSetFile.o $(BUILD)/MixtureSetEstimatorFile.o $(BUILD)/nn_kernels.o $(BUILD)/nn_api.o \
            $(BUILD)/gmm_kernels_presel.o $(BUILD)/gmm_presel.o $(BUILD)/gmm_kernels_shard.o $(BUILD)/gmm_hostio.o \
            $(BUILD)/gmm_kernels_direct.o $(BUILD)/gmm_kernels_layout.o $(BUILD)/gmm_shard.o $(BUILD)/gmm_kernels_pairs.o
DRIVER    = $(BUILD)/tests/feature_scorer_driver

REFSORT   = $(BUILD)/tests/refsort_test
CLASSLAYOUT = $(BUILD)/tests/class_layout_test

all: $(LIB) $(DRIVER) $(REFSORT) $(CLASSLAYOUT) oracle check-integration

$(BUILD)/gmm_kernels_i8.o: $(SRC)/gmm_kernels_i8.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(I8FLAGS) -c $< -o $@

$(BUILD)/gmm_kernels_f32.o: $(SRC)/gmm_kernels_f32.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(F32FLAGS) -c $< -o $@

$(BUILD)/gmm_kernels_split.o: $(SRC)/gmm_kernels_split.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(SPLITFLAGS) -c $< -o $@

# density preselection: clustering assignment + per-frame cluster selection (std::sort replay)
$(BUILD)/gmm_kernels_presel.o: $(SRC)/gmm_kernels_presel.hip $(SRC)/gmm_refsort.hh $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# reference-order float scorers (GMM_FLAG_REFERENCE_ORDER): scalar f32 ops in the reference's order
# (no SLP packing into v_pk_*_f32, which issue at a third of the scalar VOP2 rate)
$(BUILD)/gmm_kernels_direct.o: $(SRC)/gmm_kernels_direct.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -fno-slp-vectorize -c $< -o $@

# sparse best densities of (frame, mixture) pairs (gmm_best_density_pairs): the reference's scalar order
$(BUILD)/gmm_kernels_pairs.o: $(SRC)/gmm_kernels_pairs.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -fno-slp-vectorize -c $< -o $@

# density-sharded exchange keys (BASELINE config 4)
$(BUILD)/gmm_kernels_shard.o: $(SRC)/gmm_kernels_shard.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# frame-major host tables (gmm_score_host_ring with GMM_HOST_FRAME_MAJOR)
$(BUILD)/gmm_kernels_layout.o: $(SRC)/gmm_kernels_layout.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/gmm_presel.o: $(SRC)/gmm_presel.cc $(SRC)/gmm_presel.hh $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@

# hybrid-DNN scorer (include/rasr_nn.h): bf16 MFMA GEMM per layer
$(BUILD)/nn_kernels.o: $(SRC)/nn_kernels.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/nn_api.o: $(SRC)/nn_api.cc $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@

# identity of the device code: a hash of the gfx950 code objects of the GMM scorer kernels (the kernels the PMC
# summaries profiles/pmc_*.json measure), so a summary stays matched to the ISA it was collected on -- a source
# edit that leaves the code unchanged keeps the id, any code change gives a new one; bench.py uses a summary
# only for the kernels it was measured on
BUNDLER  ?= $(ROCM_PATH)/lib/llvm/bin/clang-offload-bundler
KERNEL_OBJS = $(BUILD)/gmm_kernels_i8.o $(BUILD)/gmm_kernels_f32.o $(BUILD)/gmm_kernels_split.o
$(BUILD)/kernel_id.h: $(KERNEL_OBJS)
	@for o in $(KERNEL_OBJS); do objcopy -O binary --only-section=.hip_fatbin $$o $$o.fatbin && \
	     $(BUNDLER) --unbundle --type=o --input=$$o.fatbin --targets=hipv4-amdgcn-amd-amdhsa--$(ARCH) \
	     --output=$$o.$(ARCH) || exit 1; done
	@echo "#define GMM_KERNEL_ID \"$$(cat $(addsuffix .$(ARCH),$(KERNEL_OBJS)) | sha256sum | cut -c1-16)\"" > $@

$(BUILD)/gmm_api.o: $(SRC)/gmm_api.cc $(HDRS) $(BUILD)/kernel_id.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HOSTFLAGS) -I$(BUILD) -c $< -o $@

$(BUILD)/gmm_hostio.o: $(SRC)/gmm_hostio.cc $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HOSTFLAGS) -pthread -c $< -o $@

# density shard plan (gmm_scorer_create_sharded, gmm_density_shard_plan)
$(BUILD)/gmm_shard.o: $(SRC)/gmm_shard.cc $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@

$(BUILD)/gmm_prepare.o: $(SRC)/gmm_prepare.cc $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@

$(BUILD)/GpuFeatureScorer.o: $(SRC)/host/GpuFeatureScorer.cc $(HDRS)
	@mkdir -p $(BUILD)
	g++ $(HOSTFLAGS) -c $< -o $@

$(BUILD)/MixtureSetFile.o: $(SRC)/host/MixtureSetFile.cc $(HDRS)
	@mkdir -p $(BUILD)
	g++ $(HOSTFLAGS) -c $< -o $@

$(BUILD)/MixtureSetEstimatorFile.o: $(SRC)/host/MixtureSetEstimatorFile.cc $(HDRS)
	@mkdir -p $(BUILD)
	g++ $(HOSTFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -lz -pthread -ldl

# host check of the score-only layout against the SCORE_ONLY kernel's arithmetic (no GPU)
$(CLASSLAYOUT): tests/cpp/class_layout_test.cc $(BUILD)/gmm_prepare.o $(HDRS)
	@mkdir -p $(BUILD)/tests
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@.o
	$(HIPCC) -o $@ $@.o $(BUILD)/gmm_prepare.o

# host pin of the GPU std::sort replay (gmm_refsort.hh) against this image's std::sort
$(REFSORT): tests/cpp/refsort_test.cc $(SRC)/gmm_refsort.hh
	@mkdir -p $(BUILD)/tests
	g++ -std=c++17 -O2 -Wall -o $@ $<

$(DRIVER): tests/cpp/feature_scorer_driver.cc $(LIB) $(HDRS)
	@mkdir -p $(BUILD)/tests
	g++ $(HOSTFLAGS) -o $@ $< -L$(LIBDIR) -lrasr_gmm -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

oracle:
	$(MAKE) -C oracle

# The RASR-side adapter (integration/rasr/Mm/GpuFeatureScorer.{hh,cc}) compiled -fsyntax-only against the
# reference's own headers with the reference's flags (config/cc-gcc.make:26-29).  Core/Utility.hh includes the
# make-generated Modules.hh, so a one-line stand-in (MODULE_MM_BATCH, as src/Mm/Makefile:70-75 builds it) is
# written under build/ for this check only; it pins no parity and nothing is linked.  Skipped where the
# reference tree is absent (the GPU box).
RASR_SRC ?= /root/reference/src
check-integration: integration/rasr/Mm/GpuFeatureScorer.cc integration/rasr/Mm/GpuFeatureScorer.hh $(SRC)/host/GpuFeatureScorer.hh \
                   integration/rasr/Nn/GpuBatchFeatureScorer.cc integration/rasr/Nn/GpuBatchFeatureScorer.hh \
                   integration/rasr/Nn/GpuBatchFeatureScorerNetwork.cc include/rasr_nn.h
	@if [ -d "$(RASR_SRC)/Mm" ]; then \
	    mkdir -p $(BUILD)/rasr_check && printf '#pragma once\n#define MODULE_MM_BATCH\n' > $(BUILD)/rasr_check/Modules.hh && \
	    g++ -std=gnu++0x -fsyntax-only -funsigned-char -fno-exceptions -Wall -DPROC_x86_64 -DOS_linux \
	        -DARCH_linux_x86_64 -D_GNU_SOURCE -I$(BUILD)/rasr_check -I$(RASR_SRC) -I/usr/include/libxml2 -Iinclude \
	        -I$(SRC) integration/rasr/Mm/GpuFeatureScorer.cc && \
	    g++ -std=gnu++0x -fsyntax-only -funsigned-char -fno-exceptions -Wall -DPROC_x86_64 -DOS_linux \
	        -DARCH_linux_x86_64 -D_GNU_SOURCE -I$(BUILD)/rasr_check -I$(RASR_SRC) -I/usr/include/libxml2 \
	        -Iinclude integration/rasr/Nn/GpuBatchFeatureScorer.cc && \
	    echo "check-integration: adapters compile against $(RASR_SRC) (Mm; Nn protocol unit -- its network unit" \
	         "includes Math/Blas.hh -> <cblas.h>, absent from this image, and is not checked)"; \
	else echo "check-integration: $(RASR_SRC) absent, skipped"; fi

# The RASR-side adapter LINKED and RUN on the CPU (test infrastructure): integration/rasr/Mm/GpuFeatureScorer.cc and
# the real host classes (rasr_amd/csrc/host/GpuFeatureScorer.cc) inside test doubles of RASR's plugin machinery
# (tests/rasr_harness/include, see its README), over an oracle-backed stand-in of the C-ABI; driven through the
# factory, FeatureScorerScaling, the recognizer and the score-dump call sequences (tests/rasr_harness/harness.cc).
HARNESS = $(BUILD)/tests/rasr_adapter_harness
$(HARNESS): tests/rasr_harness/harness.cc tests/rasr_harness/gmm_standin.cc integration/rasr/Mm/GpuFeatureScorer.cc \
            integration/rasr/Mm/GpuFeatureScorer.hh $(SRC)/host/GpuFeatureScorer.cc $(SRC)/host/GpuFeatureScorer.hh \
            $(wildcard tests/rasr_harness/include/*/*.hh) | oracle
	@mkdir -p $(BUILD)/tests
	g++ -std=c++17 -O1 -Wall -Wno-unused-variable -Itests/rasr_harness/include -Iinclude -I$(SRC) -o $@ \
	    tests/rasr_harness/harness.cc tests/rasr_harness/gmm_standin.cc integration/rasr/Mm/GpuFeatureScorer.cc \
	    $(SRC)/host/GpuFeatureScorer.cc -Loracle/_build -lgmm_oracle -Wl,-rpath,'$$ORIGIN/../../oracle/_build' -lm -pthread

# The hybrid-DNN adapter (all three integration/rasr/Nn files) linked and run the same way: test doubles of the Nn
# network, prior and class-label classes (tests/rasr_harness/include/Nn), over an f32 stand-in of the NN C-ABI (CPU)
# or the product library (GPU build, run by tests/test_nn_integration.py -m gpu)
NN_ADAPTER = integration/rasr/Nn/GpuBatchFeatureScorer.cc integration/rasr/Nn/GpuBatchFeatureScorerNetwork.cc
NN_HARNESS_DEPS = tests/rasr_harness/nn_harness.cc $(NN_ADAPTER) integration/rasr/Nn/GpuBatchFeatureScorer.hh \
                  include/rasr_nn.h $(wildcard tests/rasr_harness/include/*/*.hh)
NN_HARNESS_FLAGS = -std=c++17 -O1 -Wall -Wno-unused-variable -Itests/rasr_harness/include -Itests/rasr_harness/include/Nn -Iinclude
NN_HARNESS = $(BUILD)/tests/rasr_nn_harness
$(NN_HARNESS): $(NN_HARNESS_DEPS) tests/rasr_harness/nn_standin.cc
	@mkdir -p $(BUILD)/tests
	g++ $(NN_HARNESS_FLAGS) -o $@ tests/rasr_harness/nn_harness.cc $(NN_ADAPTER) tests/rasr_harness/nn_standin.cc -lm
NN_HARNESS_GPU = $(BUILD)/tests/rasr_nn_harness_gpu
$(NN_HARNESS_GPU): $(NN_HARNESS_DEPS) $(LIB)
	@mkdir -p $(BUILD)/tests
	g++ $(NN_HARNESS_FLAGS) -DHARNESS_PRODUCT -o $@ tests/rasr_harness/nn_harness.cc $(NN_ADAPTER) \
	    -L$(LIBDIR) -lrasr_gmm -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -lm -pthread

check-integration-link: $(HARNESS) $(NN_HARNESS)
	$(HARNESS)

# The same adapter + harness over the PRODUCT library (librasr_gmm.so: the HIP kernels and the host classes inside
# it); the oracle is linked as the checker.  Built here, run on the GPU by tests/test_integration.py (-m gpu).
HARNESS_GPU = $(BUILD)/tests/rasr_adapter_harness_gpu
$(HARNESS_GPU): tests/rasr_harness/harness.cc integration/rasr/Mm/GpuFeatureScorer.cc integration/rasr/Mm/GpuFeatureScorer.hh \
                $(SRC)/host/GpuFeatureScorer.hh $(wildcard tests/rasr_harness/include/*/*.hh) $(LIB) | oracle
	@mkdir -p $(BUILD)/tests
	g++ -std=c++17 -O1 -Wall -Wno-unused-variable -DHARNESS_PRODUCT -Itests/rasr_harness/include -Iinclude -I$(SRC) -o $@ \
	    tests/rasr_harness/harness.cc integration/rasr/Mm/GpuFeatureScorer.cc \
	    -L$(LIBDIR) -lrasr_gmm -Loracle/_build -lgmm_oracle \
	    -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,'$$ORIGIN/../../oracle/_build' -lm -pthread

# the harness binaries (variables defined above): built with everything else, so they travel to the GPU box
all: $(HARNESS_GPU) $(NN_HARNESS) $(NN_HARNESS_GPU)

clean:
	rm -rf $(BUILD) $(LIBDIR)
	$(MAKE) -C oracle clean

# make -s print-VAR: a variable's value (scripts/build_variants.sh takes the per-TU kernel flags from here)
print-%:
	@echo '$($*)'

.PHONY: all oracle clean check-integration check-integration-link
