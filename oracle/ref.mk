# TEST INFRASTRUCTURE ONLY: builds oracle/_ref/gbref, a harness around the
# reference's own PosdbTable / TopTree / RdbList::merge_r compiled from the
# UNMODIFIED sources under /root/reference.  Output goes only to oracle/_ref/
# (git-ignored; it travels to the GPU box with the tree, where the bench's
# cpu_baseline leg may time it).  Nothing is copied into the repo and no
# reference file is edited or replaced.
#
#   make -f oracle/ref.mk -j8        (only where /root/reference exists)
#
# Recipe:
#  * units = the gb binary's own object list (OBJS, Makefile:11-68), compiled
#    with the reference's flags (Makefile:101,433-434: -O2 gnu++98
#    -fpermissive -DPTHREADS) by g++ directly -- the reference's build system
#    is not run.
#  * Mem.cpp: g++ 11 rejects its operator new redeclaration (no throw() spec
#    vs Mem.h:219); clang accepts it with a warning, so this one unit is
#    compiled with amdclang++ (same Itanium ABI and libstdc++).
#  * Xml.cpp (Xml.cpp:1202) and Unicode.cpp (Unicode.cpp:1746-1747) are
#    rejected by both compilers as written (ordered pointer/zero compares),
#    and geo_ip_table.cpp is absent (Makefile:60); none is on the query or
#    merge path, so they are left out.  gb's global constructors are not run
#    (.init_array is dropped from each unit): they construct server
#    subsystems (Conf holds an Xml, Conf.h:771; Posdb holds an Rdb ...), and
#    the harness calls the path's own initialisers (Mem::init, hashinit)
#    instead.  Unresolved references stay at address 0
#    (--unresolved-symbols=ignore-all): reaching one faults loudly, and the
#    harness prints the caller.
REF      ?= /root/reference
OUT      := oracle/_ref
OBJ      := $(OUT)/obj
CXX      ?= g++
CC       ?= gcc
CLANGXX  ?= /opt/rocm/llvm/bin/clang++
REFFLAGS := -O2 -g0 -w -pipe -fno-pie -fno-stack-protector -DPTHREADS -std=gnu++98 -fpermissive -I$(REF)

GB_OBJS  := $(shell sed -n '/^OBJS *=/,/Version\.o/p' $(REF)/Makefile | grep -o '[A-Za-z0-9_]*\.o')
SKIP     := Xml.o Unicode.o geo_ip_table.o dlstubs.o
UNITS    := $(filter-out $(SKIP),$(GB_OBJS))
OBJS     := $(addprefix $(OBJ)/,$(UNITS))

all: $(OUT)/gbref $(OUT)/gbref_gpu

# compile, then drop the unit's global constructors/destructors
define strip_init
objcopy --remove-section=.init_array --remove-section=.fini_array $@
endef

$(OBJ)/Mem.o: $(REF)/Mem.cpp
	@mkdir -p $(OBJ)
	$(CLANGXX) $(REFFLAGS) -Wno-everything -c $< -o $@
	$(strip_init)

$(OBJ)/%.o: $(REF)/%.cpp
	@mkdir -p $(OBJ)
	$(CXX) $(REFFLAGS) -c $< -o $@
	$(strip_init)

$(OBJ)/%.o: $(REF)/%.c
	@mkdir -p $(OBJ)
	$(CC) -O2 -w -fno-pie -I$(REF) -c $< -o $@
	$(strip_init)

$(OBJ)/ref_harness.o: oracle/ref_harness.cpp oracle/posdb_oracle.h
	@mkdir -p $(OBJ)
	$(CXX) $(REFFLAGS) -Ioracle -c $< -o $@

$(OUT)/gbref: $(OBJS) $(OBJ)/ref_harness.o
	$(CXX) -no-pie -o $@ $^ -Wl,--unresolved-symbols=ignore-all -lm -lpthread -lssl -lcrypto -lz

# gbref_gpu: the same harness with INTEGRATION.md's adapter (generated into
# $(OUT)/adapter.cpp by oracle/adapter_tu.py) and libgbgpu.so linked in; op 4
# runs the adapter inside the reference's own Msg39 sequence
# (tests/test_adapter.py, on the GPU box).  Mem.cpp's global operator
# new/delete (Mem.cpp:175-360: g_mem accounting) would otherwise serve every
# C++ allocation of the HIP runtime too, static initialisers before main
# included; in this binary they are local to Mem's own unit (objcopy
# --localize-symbol on a copy of its object), so every allocation pairs
# with libstdc++'s.
GBGPU_LIB := open-source-search-engine_amd/lib
NEWDEL   := _Znwm _Znam _ZdlPv _ZdaPv _ZnwmRKSt9nothrow_t _ZnamRKSt9nothrow_t

$(OUT)/adapter.cpp: INTEGRATION.md oracle/adapter_tu.py
	@mkdir -p $(OUT)
	python3 oracle/adapter_tu.py INTEGRATION.md > $@

$(OBJ)/adapter.o: $(OUT)/adapter.cpp include/gbgpu.h
	@mkdir -p $(OBJ)
	$(CXX) $(REFFLAGS) -Iinclude -c $< -o $@

$(OBJ)/Mem_local.o: $(OBJ)/Mem.o
	objcopy $(addprefix --localize-symbol=,$(NEWDEL)) $< $@

$(OUT)/gbref_gpu: $(filter-out $(OBJ)/Mem.o,$(OBJS)) $(OBJ)/Mem_local.o $(OBJ)/ref_harness.o $(OBJ)/adapter.o \
                  $(GBGPU_LIB)/libgbgpu.so
	$(CXX) -no-pie -o $@ $(filter %.o,$^) -Wl,--unresolved-symbols=ignore-all -L$(GBGPU_LIB) -lgbgpu \
	  -Wl,-rpath,'$$ORIGIN/../../$(GBGPU_LIB)' -lm -lpthread -lssl -lcrypto -lz

clean:
	rm -rf $(OUT)

.PHONY: all clean
