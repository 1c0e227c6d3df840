# Build of the MI355X backend (gfx950) and of the CPU oracle.
#   make            -> hpx_amd/libhpxhip.so + oracle/_build/liboracle.so
#   make lib        -> the HIP library only
#   make oracle     -> the oracle only (g++, no ROCm needed)
#   make cxxtests   -> C++ tests of the header-only HPX-API layer
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
BUILD    := build

# --offload-compress: the gfx950 code objects are stored compressed (the HIP
# runtime inflates them at load): the library is ~3x smaller on disk, which
# keeps the tree each GPU run ships small
HIPFLAGS := -O3 --offload-arch=$(ARCH) -fPIC -std=c++17 -ffp-contract=off --offload-compress \
            -Wall -Wno-unused-result -Wno-unused-function -Iinclude
LIB      := hpx_amd/libhpxhip.so
KSRC     := runtime elementwise reduce scan copy_if sort merge stencil
KOBJ     := $(KSRC:%=$(BUILD)/csrc/%.o)
KHDR     := $(wildcard hpx_amd/csrc/*.hpp) $(wildcard include/hpxhip/kernels/*.hpp) include/hpxhip.h

ORACLE   := oracle/_build/liboracle.so
OFLAGS   := -O2 -fPIC -std=c++17 -ffp-contract=off -Wall -pthread

.PHONY: all lib oracle clean cxxtests oracle-sanitize mw-variants

# C++ tests of include/hpx (plain g++ host code linked to the C ABI library)
CXXT     := compute_api algorithms_known_answer stream_hip for_loop_merge stencil_partitioned call_overhead exception_list futures
CXXTBIN  := $(CXXT:%=tests/cxx/bin/%)
CXXHDR   := $(shell find include -name '*.hpp') include/hpxhip.h
TFLAGS   := -O2 -std=c++17 -Wall -Wextra -Wno-unused-parameter -pthread -Iinclude
TLINK    := -Lhpx_amd -lhpxhip -Wl,-rpath,'$$ORIGIN/../../../hpx_amd' -Wl,-rpath,/opt/rocm/lib \
            -Wl,-rpath-link,/opt/rocm/lib

all: lib oracle mw-variants

lib: $(LIB)
oracle: $(ORACLE)

$(BUILD)/csrc/%.o: hpx_amd/csrc/%.hip $(KHDR)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(KOBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(KOBJ)

# merge.hip: the multiway merge (k_mw_merge) must not spill SGPRs.  An
# earlier form of it, built at 8 waves per SIMD with 20-22 SGPR spills, was
# miscompiled (registers of live outputs reused as temporaries in a divergent
# branch: float64 keys written in their ordered-bit form; DESIGN.md (e),
# profiles/r06_mw_merge_miscompile.txt).  The build refuses a k_mw_merge
# instantiation with spills instead of shipping one.
define mw_spill_guard
	@awk '/Function Name:/ {k = ($$0 ~ /k_mw_merge/)} k && /SGPRs Spill: [1-9]/ {bad = 1; print} \
	     END {if (bad) {print "merge.hip: k_mw_merge spills SGPRs (see Makefile)"; exit 1}}' $(1)
endef
$(BUILD)/csrc/merge.o: hpx_amd/csrc/merge.hip $(KHDR)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -Rpass-analysis=kernel-resource-usage -c $< -o $@ 2> $(BUILD)/csrc/merge.usage || \
	    (cat $(BUILD)/csrc/merge.usage; rm -f $@; exit 1)
	$(call mw_spill_guard,$(BUILD)/csrc/merge.usage) || (rm -f $@; exit 1)

# Variant builds of the multiway merge kept in the standing test matrix
# (tests/test_gpu_merge_sort.py::test_merge_runs_variant_builds):
# 512-thread tasks, and 256 threads at the default occupancy bound.  Each is
# library of its own (hpx_amd/variants/<name>/), the shipped objects but merge.o.
MWVAR    := mw512 mwminw4
MWVAR_mw512   := -DHPXHIP_MW_THREADS=512 -DHPXHIP_MW_MINW=4
MWVAR_mwminw4 := -DHPXHIP_MW_MINW=4
mw-variants: $(MWVAR:%=hpx_amd/variants/%/libhpxhip.so)
hpx_amd/variants/%/libhpxhip.so: hpx_amd/csrc/merge.hip $(filter-out $(BUILD)/csrc/merge.o,$(KOBJ)) $(KHDR)
	@mkdir -p $(dir $@) $(BUILD)/variants/$*
	$(HIPCC) $(HIPFLAGS) $(MWVAR_$*) -Rpass-analysis=kernel-resource-usage -c $< -o $(BUILD)/variants/$*/merge.o \
	    2> $(BUILD)/variants/$*/merge.usage || (cat $(BUILD)/variants/$*/merge.usage; exit 1)
	$(call mw_spill_guard,$(BUILD)/variants/$*/merge.usage)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(filter-out $(BUILD)/csrc/merge.o,$(KOBJ)) \
	    $(BUILD)/variants/$*/merge.o

$(ORACLE): oracle/oracle.cpp oracle/oracle.h
	@mkdir -p $(dir $@)
	$(CXX) $(OFLAGS) -shared -o $@ oracle/oracle.cpp

# The oracle under ASan + UBSan (host code only)
SANFLAGS := -O0 -std=c++17 -ffp-contract=off -pthread -fsanitize=address,undefined -fno-sanitize-recover=all
oracle-sanitize: tests/cxx/bin/oracle_sanitize
tests/cxx/bin/oracle_sanitize: tests/cxx/oracle_sanitize.cpp oracle/oracle.cpp oracle/oracle.h include/hpxhip.h
	@mkdir -p $(dir $@)
	$(CXX) $(SANFLAGS) tests/cxx/oracle_sanitize.cpp oracle/oracle.cpp -o $@

# ... and the hipcc-compiled ones (device closures, HPX_HOST_DEVICE lambdas)
HIPT     := device_closures partitioned_vector closure_algorithms closure_timing dataflow_stencil bench_targets
HIPTBIN  := $(HIPT:%=tests/cxx/bin/%)
HTFLAGS  := -O2 -std=c++17 --offload-arch=$(ARCH) --offload-compress -Wall -Wno-unused-parameter -Iinclude

cxxtests: $(CXXTBIN) $(HIPTBIN)

tests/cxx/bin/%: tests/cxx/%.cpp $(CXXHDR) $(LIB)
	@mkdir -p $(dir $@)
	$(CXX) $(TFLAGS) $< -o $@ $(TLINK)

tests/cxx/bin/%: tests/cxx/%.hip $(CXXHDR) $(LIB)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HTFLAGS) $< -o $@ $(TLINK)

# the dataflow stencil checks itself against the oracle (test infrastructure)
tests/cxx/bin/dataflow_stencil: tests/cxx/dataflow_stencil.hip $(CXXHDR) $(LIB) $(ORACLE)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HTFLAGS) $< -o $@ $(TLINK) -Loracle/_build -loracle -Wl,-rpath,'$$ORIGIN/../../../oracle/_build'

clean:
	rm -rf $(BUILD) $(LIB) oracle/_build tests/cxx/bin hpx_amd/variants
