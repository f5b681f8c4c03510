# Build of the MI355X-native library (gfx950 only), the drivers and the oracle.
#   make            -> nonlinear-solvers_amd/lib/libnls_amd.so + drivers + oracle
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := nonlinear-solvers_amd
CSRC     := $(PKG)/csrc
BUILD    := $(PKG)/build
LIBDIR   := $(PKG)/lib
BINDIR   := $(PKG)/bin
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -I$(CSRC) -Wall
LDFLAGS  := -shared -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

LIB      := $(LIBDIR)/libnls_amd.so
STENCIL  := iso2 iso3 ani2 ani3
OBJS     := $(BUILD)/nls_kernels.o $(BUILD)/nls_api.o $(STENCIL:%=$(BUILD)/nls_stencil_%.o)
DEVHDR   := $(CSRC)/nls_device.hpp $(CSRC)/nls_kernels.hpp $(CSRC)/nls_stencil.hpp \
            $(CSRC)/nls_common.hpp $(CSRC)/nls_reduce.hpp

all: $(LIB) drivers oracle

$(BUILD) $(LIBDIR) $(BINDIR):
	mkdir -p $@

$(BUILD)/nls_kernels.o: $(CSRC)/nls_kernels.hip $(DEVHDR) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the stencil tables, one object per operator variant x dimension (parallel build)
$(BUILD)/nls_stencil_%.o: $(CSRC)/nls_stencil.hip $(DEVHDR) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DNLS_ANI=$(if $(findstring ani,$*),1,0) -DNLS_DIM=$(subst ani,,$(subst iso,,$*)) \
	  -DNLS_TABLE=stencil_table_$* -c $< -o $@

$(BUILD)/nls_api.o: $(CSRC)/nls_api.cpp $(CSRC)/nls_device.hpp $(CSRC)/nls_kernels.hpp include/nls.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(OBJS) | $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) $(OBJS) $(LDFLAGS) -o $@

drivers: $(LIB)
	@if [ -f $(PKG)/drivers/Makefile ]; then $(MAKE) -C $(PKG)/drivers; fi

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) $(LIBDIR) $(BINDIR)
	$(MAKE) -C oracle clean

.PHONY: all drivers oracle clean
