# Top-level build: the MI355X scorer library, the C++ host-side scorer classes,
# the C++ test drivers, and the (test-only) oracle.  No cmake; hipcc for gfx950.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
BUILD     = build
LIBDIR    = rasr_amd/lib
HIPFLAGS  = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result
HOSTFLAGS = -O2 -std=c++17 -fPIC -ffp-contract=off -Wall

SRC       = rasr_amd/csrc
HDRS      = include/rasr_gmm.h $(SRC)/gmm_prepare.hh $(SRC)/gmm_kernels.hh

LIB       = $(LIBDIR)/librasr_gmm.so
OBJS      = $(BUILD)/gmm_kernels.o $(BUILD)/gmm_api.o $(BUILD)/gmm_prepare.o

all: $(LIB) oracle

$(BUILD)/gmm_kernels.o: $(SRC)/gmm_kernels.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/gmm_api.o: $(SRC)/gmm_api.cc $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@

$(BUILD)/gmm_prepare.o: $(SRC)/gmm_prepare.cc $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) $(LIBDIR)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
