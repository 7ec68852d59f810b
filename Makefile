# Builds the MI355X backend (librnsntt.so, gfx950) and the CPU oracle
# (liboracle.so, test infrastructure).  `python -c "import __graft_entry__ as g;
# g.build()"` runs the same commands.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := toy-heaan-ckks_amd
CSRC     := $(PKG)/csrc
LIBDIR   := $(PKG)/lib
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
CFLAGS   := -O2 -fPIC -std=c11 -Wall -pthread

all: $(LIBDIR)/librnsntt.so $(LIBDIR)/isa_check.ok oracle/liboracle.so

# Every header each translation unit includes, transitively (a CPU test,
# tests/test_abi_cpu.py::test_makefile_dependencies_match_includes, diffs
# these lists against the sources' #include lines).
DEP_rnt_kernels := $(CSRC)/rnt_internal.hpp $(CSRC)/rnt_modarith.hpp $(CSRC)/rnt_device.hpp
DEP_rnt_plane   := $(CSRC)/rnt_internal.hpp $(CSRC)/rnt_modarith.hpp $(CSRC)/rnt_device.hpp $(CSRC)/rnt_bfly4.hpp
DEP_rnt_mfma    := $(CSRC)/rnt_internal.hpp $(CSRC)/rnt_hostmath.hpp $(CSRC)/rnt_modarith.hpp $(CSRC)/rnt_device.hpp
DEP_rnt_encode  := $(CSRC)/rnt_internal.hpp
DEP_rnt_sample  := $(CSRC)/rnt_internal.hpp $(CSRC)/rnt_modarith.hpp
DEP_rnt_api     := $(CSRC)/rnt_internal.hpp $(CSRC)/rnt_hostmath.hpp include/rnsntt.h

OBJS := $(LIBDIR)/rnt_kernels.o $(LIBDIR)/rnt_plane.o $(LIBDIR)/rnt_mfma.o $(LIBDIR)/rnt_encode.o \
        $(LIBDIR)/rnt_sample.o $(LIBDIR)/rnt_api.o

$(LIBDIR)/rnt_kernels.o: $(CSRC)/rnt_kernels.hip $(DEP_rnt_kernels)
$(LIBDIR)/rnt_plane.o: $(CSRC)/rnt_plane.hip $(DEP_rnt_plane)
$(LIBDIR)/rnt_mfma.o: $(CSRC)/rnt_mfma.hip $(DEP_rnt_mfma)
$(LIBDIR)/rnt_encode.o: $(CSRC)/rnt_encode.hip $(DEP_rnt_encode)
$(LIBDIR)/rnt_sample.o: $(CSRC)/rnt_sample.hip $(DEP_rnt_sample)
$(LIBDIR)/rnt_api.o: $(CSRC)/rnt_api.cpp $(DEP_rnt_api)

$(OBJS):
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/librnsntt.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@

# The ISA hazard check build() runs (tools/isa_check.py, DESIGN.md §3 "MFMA
# hazards"): every kernel of every object, back edges followed; a finding
# fails the build, and the stamp is written only when it passes.
$(LIBDIR)/isa_check.ok: $(OBJS) tools/isa_check.py
	python3 tools/isa_check.py $(OBJS)
	echo ok > $@

oracle/liboracle.so: oracle/oracle.c oracle/oracle.h
	gcc $(CFLAGS) -shared oracle/oracle.c -o $@

# ASan + UBSan variants of the oracle and of librnsntt's host code, and the
# CPU tests run under them; log in profiles/rNN_sanitizer_cpu.log
# (tools/sanitize.sh names the round)
asan:
	tools/sanitize.sh

clean:
	rm -f $(LIBDIR)/*.o $(LIBDIR)/*.so $(LIBDIR)/isa_check.ok oracle/liboracle.so

.PHONY: all clean asan
