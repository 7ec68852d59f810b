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

all: $(LIBDIR)/librnsntt.so oracle/liboracle.so

$(LIBDIR)/rnt_kernels.o: $(CSRC)/rnt_kernels.hip $(CSRC)/rnt_internal.hpp $(CSRC)/rnt_modarith.hpp $(CSRC)/rnt_device.hpp
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/rnt_plane.o: $(CSRC)/rnt_plane.hip $(CSRC)/rnt_internal.hpp $(CSRC)/rnt_modarith.hpp $(CSRC)/rnt_device.hpp
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/rnt_mfma.o: $(CSRC)/rnt_mfma.hip $(CSRC)/rnt_internal.hpp $(CSRC)/rnt_hostmath.hpp
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/rnt_encode.o: $(CSRC)/rnt_encode.hip $(CSRC)/rnt_internal.hpp
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/rnt_sample.o: $(CSRC)/rnt_sample.hip $(CSRC)/rnt_internal.hpp $(CSRC)/rnt_modarith.hpp
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/rnt_api.o: $(CSRC)/rnt_api.cpp $(CSRC)/rnt_internal.hpp $(CSRC)/rnt_hostmath.hpp include/rnsntt.h
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/librnsntt.so: $(LIBDIR)/rnt_kernels.o $(LIBDIR)/rnt_plane.o $(LIBDIR)/rnt_mfma.o $(LIBDIR)/rnt_encode.o $(LIBDIR)/rnt_sample.o $(LIBDIR)/rnt_api.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@

oracle/liboracle.so: oracle/oracle.c oracle/oracle.h
	gcc $(CFLAGS) -shared oracle/oracle.c -o $@

# ASan + UBSan variants of the oracle and of librnsntt's host code, and the
# CPU tests run under them; log in profiles/r03_sanitizer_cpu.log
asan:
	tools/sanitize.sh

clean:
	rm -f $(LIBDIR)/*.o $(LIBDIR)/*.so oracle/liboracle.so

.PHONY: all clean asan
