# Build libs2c.so (HIP kernels for gfx950 + host parser/planner/generator) in-tree.
# Used by __graft_entry__.build(); also `make -j8` by hand.
HIPCC   ?= /opt/rocm/bin/hipcc
CXX     ?= g++
ARCH    ?= gfx950
SRC      = sam2consensus_amd/csrc
OUT      = sam2consensus_amd/libs2c.so
BUILD    = build
CXXFLAGS = -O3 -std=c++17 -fPIC -pthread -Wall -Wextra -Iinclude
HIPFLAGS = -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -Iinclude \
           -Wno-unused-result

all: $(OUT)

$(BUILD)/s2c_host.o: $(SRC)/s2c_host.cpp include/s2c.h | $(BUILD)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(BUILD)/s2c_synth.o: $(SRC)/s2c_synth.cpp include/s2c.h | $(BUILD)
	$(CXX) $(CXXFLAGS) -c $< -o $@

# (every kernel's resource remarks checked: a spill fails the build, scripts/check_spills.py)
$(BUILD)/%.o: $(SRC)/%.hip $(SRC)/s2c_common.h include/s2c.h scripts/check_spills.py | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -Rpass-analysis=kernel-resource-usage -c $< -o $@ 2> $(BUILD)/$*.usage || { cat $(BUILD)/$*.usage; exit 1; }
	python3 scripts/check_spills.py $(BUILD)/$*.usage || { rm -f $@; exit 1; }

KOBJ = $(BUILD)/s2c_reads.o $(BUILD)/s2c_tile.o $(BUILD)/s2c_dense.o $(BUILD)/s2c_bodies.o

$(OUT): $(BUILD)/s2c_host.o $(BUILD)/s2c_synth.o $(KOBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $^ -lz -lpthread -o $@

$(BUILD):
	mkdir -p $(BUILD)

# diagnostic build: phase clocks of k_tile_dense (S2C_LIB=libs2c_prof.so, scripts/prof_dense.py)
PROF_OUT = sam2consensus_amd/libs2c_prof.so
prof: $(BUILD)/s2c_host.o $(BUILD)/s2c_synth.o $(BUILD)/s2c_reads.o $(BUILD)/s2c_bodies.o $(SRC)/s2c_tile.hip $(SRC)/s2c_dense.hip $(SRC)/s2c_common.h
	$(HIPCC) $(HIPFLAGS) $(VDEFS) -DS2C_PROF -c $(SRC)/s2c_dense.hip -o $(BUILD)/s2c_dense_prof.o
	$(HIPCC) $(HIPFLAGS) $(VDEFS) -DS2C_PROF -c $(SRC)/s2c_tile.hip -o $(BUILD)/s2c_tile_prof.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(BUILD)/s2c_host.o $(BUILD)/s2c_synth.o $(BUILD)/s2c_reads.o $(BUILD)/s2c_bodies.o \
	  $(BUILD)/s2c_tile_prof.o $(BUILD)/s2c_dense_prof.o -lz -lpthread -o $(PROF_OUT)

# kernel resource usage (VGPR/SGPR/LDS/occupancy) and ISA for inspection
ISA_DIR ?= /tmp/s2c_isa
isa:
	mkdir -p $(ISA_DIR)
	for f in s2c_reads s2c_tile s2c_dense; do \
	  $(HIPCC) $(HIPFLAGS) -c $(SRC)/$$f.hip -o $(ISA_DIR)/$$f.o -save-temps=obj \
	    -Rpass-analysis=kernel-resource-usage 2> $(ISA_DIR)/$$f.resource_usage.txt; done

clean:
	rm -rf $(BUILD) $(OUT)

# diagnostic build: every kernel fills its workgroup's LDS with 0xA5 at entry (S2C_LIB=libs2c_poison.so;
# the GPU suite once under it shows no kernel reads LDS it did not write in that launch)
poison: $(BUILD)/s2c_host.o $(BUILD)/s2c_synth.o
	$(HIPCC) $(HIPFLAGS) -DS2C_LDS_POISON -c $(SRC)/s2c_reads.hip -o $(BUILD)/s2c_reads_poison.o
	$(HIPCC) $(HIPFLAGS) -DS2C_LDS_POISON -c $(SRC)/s2c_dense.hip -o $(BUILD)/s2c_dense_poison.o
	$(HIPCC) $(HIPFLAGS) -DS2C_LDS_POISON -c $(SRC)/s2c_tile.hip -o $(BUILD)/s2c_tile_poison.o
	$(HIPCC) $(HIPFLAGS) -DS2C_LDS_POISON -c $(SRC)/s2c_bodies.hip -o $(BUILD)/s2c_bodies_poison.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $^ $(BUILD)/s2c_reads_poison.o $(BUILD)/s2c_dense_poison.o \
	  $(BUILD)/s2c_tile_poison.o $(BUILD)/s2c_bodies_poison.o -lz -lpthread -o sam2consensus_amd/libs2c_poison.so

.PHONY: all clean isa prof variant poison

# experiment build: k_reads, k_tile_dense and k_tile with extra defines (V=name VDEFS='-D...'): libs2c_$(V).so
V ?= var
VDEFS ?=
variant: $(BUILD)/s2c_host.o $(BUILD)/s2c_synth.o $(BUILD)/s2c_bodies.o
	$(HIPCC) $(HIPFLAGS) $(VDEFS) -c $(SRC)/s2c_reads.hip -o $(BUILD)/s2c_reads_$(V).o
	$(HIPCC) $(HIPFLAGS) $(VDEFS) -c $(SRC)/s2c_dense.hip -o $(BUILD)/s2c_dense_$(V).o
	$(HIPCC) $(HIPFLAGS) $(VDEFS) -c $(SRC)/s2c_tile.hip -o $(BUILD)/s2c_tile_$(V).o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $^ $(BUILD)/s2c_reads_$(V).o $(BUILD)/s2c_dense_$(V).o $(BUILD)/s2c_tile_$(V).o -lz -lpthread -o sam2consensus_amd/libs2c_$(V).so
