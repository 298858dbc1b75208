# Build the product library (HIP, gfx950) and the CPU oracle (test infrastructure).
HIPCC     ?= /opt/rocm/bin/hipcc
ARCH      ?= gfx950
PKG       := neural_polar_decoder_amd
CSRC      := $(wildcard $(PKG)/csrc/*.hip)
CHDR      := $(wildcard $(PKG)/csrc/*.hpp) include/npd.h
HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude -I$(PKG)/csrc \
             -munsafe-fp-atomics
LIB       := $(PKG)/libnpd.so
OBJDIR    := build/obj
OBJS      := $(patsubst $(PKG)/csrc/%.hip,$(OBJDIR)/%.o,$(CSRC))

ORACLE    := oracle/liboracle.so

all: $(LIB) $(ORACLE)

lib: $(LIB)
oracle: $(ORACLE)

# per-file extras: the SC kernel never sees NaN (finite LLRs), so fmin needs no canonicalisation
EXTRA_npd_sc := -fno-honor-nans
EXTRA_npd_sc_fast := -fno-honor-nans
EXTRA_npd_scl := -fno-honor-nans

$(OBJDIR)/%.o: $(PKG)/csrc/%.hip $(CHDR)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXTRA_$*) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -Wl,--no-undefined

# Oracle: plain C, no fast-math, no FMA contraction (exact restatement of the reference's fp32 ops).
# The SCL restatement is C++ so that list pruning calls libstdc++'s std::nth_element (torch.topk's CPU path).
$(ORACLE): oracle/npd_oracle.c oracle/npd_oracle_scl.cpp oracle/npd_oracle_lse.c
	@mkdir -p build/oracle
	gcc -O2 -std=c11 -fPIC -fopenmp -ffp-contract=off -c oracle/npd_oracle.c -o build/oracle/npd_oracle.o
	g++ -O2 -std=c++17 -fPIC -fopenmp -ffp-contract=off -c oracle/npd_oracle_scl.cpp -o build/oracle/npd_oracle_scl.o
	gcc -O2 -std=c11 -fPIC -fopenmp -ffp-contract=off -c oracle/npd_oracle_lse.c -o build/oracle/npd_oracle_lse.o
	g++ -shared -fopenmp -o $@ build/oracle/npd_oracle.o build/oracle/npd_oracle_scl.o build/oracle/npd_oracle_lse.o -lm

asm: $(CSRC)
	@mkdir -p build/asm
	for f in $(CSRC); do b=$$(basename $$f .hip); $(HIPCC) $(HIPFLAGS) $$( case $$b in npd_sc*) echo -fno-honor-nans;; esac ) --cuda-device-only -S -o build/asm/$$b.s $$f; done

clean:
	rm -rf build $(LIB) $(ORACLE)

.PHONY: all lib oracle clean asm
