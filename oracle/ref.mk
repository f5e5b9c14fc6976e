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

all: $(OUT)/gbref

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

clean:
	rm -rf $(OUT)

.PHONY: all clean
