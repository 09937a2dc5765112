# Build for netc-mi355x: the host C library, the gfx950 HIP library, and the
# test-only oracle (oracle/Makefile).  Outputs stay in-tree so they travel to
# the GPU box with the repository snapshot.
#
#   make            libnetc.so + libnetc_ws_gpu.so (+ libnetc_ceiling.so) + oracle
#   make diag       instrumented builds + probes under tools/ (diagnostics only)
#   make host       libnetc.so only (no hipcc needed)
#   make asan       libnetc.so + the oracle built with ASan + UBSan, then the CPU suites
#                   that drive them (host framing, CPU mask, oracle checks) run against those
#   make clean

HIPCC      ?= /opt/rocm/bin/hipcc
CC         ?= gcc
ARCH       ?= gfx950
LIBDIR     := netc_amd/lib
CFLAGS     ?= -O3 -g -Wall -Wextra -Wno-unused-parameter -fPIC -std=gnu11 -fvisibility=default
HIPFLAGS   ?= -O3 -g -fPIC -std=c++17 --offload-arch=$(ARCH) -Wall -Wno-unused-result

HOST_SRCS  := $(wildcard netc_amd/csrc/host/*.c)
HOST_HDRS  := $(wildcard include/*.h include/*/*.h)
GPU_SRCS   := netc_amd/csrc/ws_mask_gpu.hip netc_amd/csrc/ws_frame_gpu.hip netc_amd/csrc/ws_scan_gpu.hip netc_amd/csrc/ws_ingest.hip netc_amd/csrc/ws_egress.hip \
              netc_amd/csrc/ws_mask_api.hip netc_amd/csrc/ws_hub.hip netc_amd/csrc/ws_egress_hub.hip
GPU_HDRS   := netc_amd/csrc/ws_mask_gpu.h netc_amd/csrc/gpu_util.h include/ws/mask.h include/ws/frame.h include/ws/ingest.h \
              include/ws/route.h include/ws/common.h include/ws/egress.h include/ws/hub.h include/ws/egress_hub.h

.PHONY: all host gpu oracle diag clean asan mock
all: host gpu oracle mock
mock: tests/bin/libnetc_ingest_mock.so tests/bin/ws_close_track_mock tests/bin/libnetc_hub_cpu.so tests/bin/ws_hub_server_cpu \
      tests/bin/ws_egress_hub_server_cpu tests/bin/ws_echo_server_cpu
host: $(LIBDIR)/libnetc.so tests/bin/ws_route_lookup
gpu: $(LIBDIR)/libnetc_ws_gpu.so $(LIBDIR)/libnetc_ceiling.so tests/bin/ws_gpu_epoll tests/bin/ws_egress_bench \
     tests/bin/ws_route_bench tests/bin/ws_hub_server tests/bin/ws_egress_hub_server tests/bin/ws_echo_server \
     tests/bin/ws_close_track

$(LIBDIR)/libnetc.so: $(HOST_SRCS) $(HOST_HDRS)
	@mkdir -p $(LIBDIR)
	$(CC) $(CFLAGS) -shared -o $@ $(HOST_SRCS) -lpthread -ldl

# one object per source (make -j compiles them in parallel), linked into one library
GPU_OBJS   := $(patsubst netc_amd/csrc/%.hip,build/%.o,$(GPU_SRCS))
build/%.o: netc_amd/csrc/%.hip $(GPU_HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIBDIR)/libnetc_ws_gpu.so: $(GPU_OBJS) $(LIBDIR)/libnetc.so
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(GPU_OBJS) -L$(LIBDIR) -lnetc -Wl,-rpath,'$$ORIGIN'

# measurement-only HBM stream kernels bench.py times beside the mask kernel (roofline ceilings)
$(LIBDIR)/libnetc_ceiling.so: netc_amd/csrc/ceiling.hip
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

# the GPU receive route under netc's caller contract (tests/test_gpu_epoll.py): a C program,
# epoll + TCP loopback, linked against both libraries as a netc server would be
tests/bin/ws_gpu_epoll: tests/drivers/ws_gpu_epoll.c $(LIBDIR)/libnetc_ws_gpu.so $(LIBDIR)/libnetc.so $(HOST_HDRS)
	@mkdir -p tests/bin
	$(CC) -O2 -g -Wall -std=gnu11 -Iinclude -o $@ $< -L$(LIBDIR) -lnetc_ws_gpu -lnetc -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib -lpthread -ldl

# send rates of the GPU egress ring beside the CPU ws_send_message (tools/bench_egress.py)
tests/bin/ws_egress_bench: tests/drivers/ws_egress_bench.c $(LIBDIR)/libnetc_ws_gpu.so $(LIBDIR)/libnetc.so $(HOST_HDRS)
	@mkdir -p tests/bin
	$(CC) -O2 -g -Wall -std=gnu11 -Iinclude -o $@ $< -L$(LIBDIR) -lnetc_ws_gpu -lnetc -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib -lpthread -ldl

# receive rates through ws_parse_frame over loopback TCP, netc's once-per-event loop: CPU path, GPU
# route, the reference's own parser (tools/bench_routes.py)
tests/bin/ws_route_bench: tests/drivers/ws_route_bench.c $(LIBDIR)/libnetc_ws_gpu.so $(LIBDIR)/libnetc.so $(HOST_HDRS)
	@mkdir -p tests/bin
	$(CC) -O2 -g -Wall -std=gnu11 -Iinclude -o $@ $< -L$(LIBDIR) -lnetc_ws_gpu -lnetc -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib -lpthread -ldl

# TEST ONLY: the ring's host code (ws_ingest.hip) over a host-memory mock of the HIP runtime
# (tests/mockhip), so tests/test_route_mock.py drives the ingest ring and the ws_parse_frame route
# on a machine without a GPU.  Never loaded by the product.
tests/bin/libnetc_ingest_mock.so: netc_amd/csrc/ws_ingest.hip netc_amd/csrc/ws_hub.hip netc_amd/csrc/ws_egress_hub.hip tests/mockhip/mock_gpu.cc tests/mockhip/hip/hip_runtime.h \
                                  netc_amd/csrc/ws_mask_gpu.h $(LIBDIR)/libnetc.so $(HOST_HDRS)
	@mkdir -p tests/bin
	g++ -O1 -g -std=c++17 -fPIC -shared -Wall -Wno-unused-result -Itests/mockhip -x c++ netc_amd/csrc/ws_ingest.hip netc_amd/csrc/ws_hub.hip netc_amd/csrc/ws_egress_hub.hip \
	    -x none tests/mockhip/mock_gpu.cc -L$(LIBDIR) -lnetc -Wl,-Bsymbolic -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -o $@

# many connections on one event loop, one GPU hub (tests/test_gpu_hub.py, tools/bench_hub.py)
tests/bin/ws_hub_server: tests/drivers/ws_hub_server.c $(LIBDIR)/libnetc_ws_gpu.so $(LIBDIR)/libnetc.so $(HOST_HDRS)
	@mkdir -p tests/bin
	$(CC) -O2 -g -Wall -std=gnu11 -Iinclude -o $@ $< -L$(LIBDIR) -lnetc_ws_gpu -lnetc -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib -lpthread -ldl

# an echo server in netc's shape, GPU both ways (receive hub in, egress hub out)
tests/bin/ws_echo_server: tests/drivers/ws_echo_server.c $(LIBDIR)/libnetc_ws_gpu.so $(LIBDIR)/libnetc.so $(HOST_HDRS)
	@mkdir -p tests/bin
	$(CC) -O2 -g -Wall -std=gnu11 -Iinclude -o $@ $< -L$(LIBDIR) -lnetc_ws_gpu -lnetc -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib -lpthread -ldl

# the send side: many connections answered from one loop through one GPU egress hub
# (tests/test_gpu_egress_hub.py, tools/bench_hub.py --send)
tests/bin/ws_egress_hub_server: tests/drivers/ws_egress_hub_server.c $(LIBDIR)/libnetc_ws_gpu.so $(LIBDIR)/libnetc.so $(HOST_HDRS)
	@mkdir -p tests/bin
	$(CC) -O2 -g -Wall -std=gnu11 -Iinclude -o $@ $< -L$(LIBDIR) -lnetc_ws_gpu -lnetc -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib -lpthread -ldl

# close() on routed sockets in a process linked as netc links libnetc.so (tests/test_close_track.py):
# against the GPU library, and against the mock (CPU suite)
tests/bin/ws_close_track: tests/drivers/ws_close_track.c $(LIBDIR)/libnetc_ws_gpu.so $(LIBDIR)/libnetc.so $(HOST_HDRS)
	@mkdir -p tests/bin
	$(CC) -O2 -g -Wall -std=gnu11 -Iinclude -o $@ $< -L$(LIBDIR) -lnetc_ws_gpu -lnetc -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib -lpthread -ldl
tests/bin/ws_close_track_mock: tests/drivers/ws_close_track.c tests/bin/libnetc_ingest_mock.so $(LIBDIR)/libnetc.so $(HOST_HDRS)
	$(CC) -O2 -g -Wall -std=gnu11 -Iinclude -o $@ $< -Ltests/bin -lnetc_ingest_mock -L$(LIBDIR) -lnetc \
	    -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -lpthread -ldl

# MEASUREMENT CONTROL ONLY ("hubcpu" legs of tools/bench_hub.py): the hubs' and rings' host code with
# the device work done on the host (tests/mockhip; netc_ws_mask for the XOR, libnetc's header walk),
# at -O3, and the server drivers linked to it -- the same batching and syscalls as the GPU legs, so
# the difference between "hub" and "hubcpu" is what the GPU itself adds or costs.  Never the product.
tests/bin/libnetc_hub_cpu.so: netc_amd/csrc/ws_ingest.hip netc_amd/csrc/ws_hub.hip netc_amd/csrc/ws_egress_hub.hip tests/mockhip/mock_gpu.cc \
                              tests/mockhip/hip/hip_runtime.h netc_amd/csrc/ws_mask_gpu.h $(LIBDIR)/libnetc.so $(HOST_HDRS)
	@mkdir -p tests/bin
	g++ -O3 -g -std=c++17 -fPIC -shared -Wall -Wno-unused-result -Itests/mockhip -x c++ netc_amd/csrc/ws_ingest.hip netc_amd/csrc/ws_hub.hip netc_amd/csrc/ws_egress_hub.hip \
	    -x none tests/mockhip/mock_gpu.cc -L$(LIBDIR) -lnetc -Wl,-Bsymbolic -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -o $@
tests/bin/%_cpu: tests/drivers/%.c tests/bin/libnetc_hub_cpu.so $(LIBDIR)/libnetc.so $(HOST_HDRS)
	$(CC) -O2 -g -Wall -std=gnu11 -Iinclude -o $@ $< -Ltests/bin -lnetc_hub_cpu -L$(LIBDIR) -lnetc \
	    -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -lpthread -ldl

# the per-call cost of an attached socket's route lookups, close-tracked or fstat-checked (host only)
tests/bin/ws_route_lookup: tests/drivers/ws_route_lookup.c $(LIBDIR)/libnetc.so $(HOST_HDRS)
	@mkdir -p tests/bin
	$(CC) -O2 -g -Wall -std=gnu11 -Iinclude -o $@ $< -L$(LIBDIR) -lnetc -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -lpthread -ldl

oracle:
	$(MAKE) -C oracle

clean:
	rm -f $(LIBDIR)/*.so build/*.o tests/bin/ws_gpu_epoll tests/bin/ws_egress_bench tests/bin/ws_route_bench \
	    tests/bin/libnetc_ingest_mock.so tests/bin/ws_hub_server tests/bin/ws_egress_hub_server tests/bin/ws_echo_server \
	    tests/bin/ws_close_track tests/bin/ws_close_track_mock tests/bin/libnetc_hub_cpu.so tests/bin/*_cpu \
	    tests/bin/ws_route_lookup
	$(MAKE) -C oracle clean

# diagnostics (tools/, not part of the product)
diag: tools/libdiag_stream.so tools/libnetc_ws_gpu_stamps.so tools/libnetc_ws_gpu_checks.so tools/libscan_k1only.so \
      tools/libscan_k1exp.so diag/libnetc_ws_gpu_trace.so diag/libnetc_ws_gpu_nofix.so
tools/libdiag_stream.so: tools/diag_stream.hip
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<
tools/libnetc_ws_gpu_stamps.so: $(GPU_SRCS) $(GPU_HDRS) $(LIBDIR)/libnetc.so
	$(HIPCC) $(HIPFLAGS) -DNETC_MASK_STAMPS -DNETC_SCAN_STAMPS -shared -o $@ $(GPU_SRCS) -L$(LIBDIR) -lnetc -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'
tools/libnetc_ws_gpu_checks.so: $(GPU_SRCS) $(GPU_HDRS) $(LIBDIR)/libnetc.so
	$(HIPCC) $(HIPFLAGS) -DNETC_ENC_CHECKS -shared -o $@ $(GPU_SRCS) -L$(LIBDIR) -lnetc -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'
tools/libscan_k1only.so: $(GPU_SRCS) $(GPU_HDRS) $(LIBDIR)/libnetc.so
	$(HIPCC) $(HIPFLAGS) -DNETC_SCAN_K1_ONLY -shared -o $@ $(GPU_SRCS) -L$(LIBDIR) -lnetc -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'
# one-pass scan progress words in host-mapped memory (tools/scan_probe.py); diag/ travels to the GPU box
diag/libnetc_ws_gpu_trace.so: $(GPU_SRCS) $(GPU_HDRS) $(LIBDIR)/libnetc.so
	@mkdir -p diag
	$(HIPCC) $(HIPFLAGS) -DNETC_SCAN_TRACE -shared -o $@ $(GPU_SRCS) -L$(LIBDIR) -lnetc -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'
# the frame assembly without its header fixups (wrong wire bytes: counter attribution only,
# tools/pmc_encode_fixups.sh)
diag/libnetc_ws_gpu_nofix.so: $(GPU_SRCS) $(GPU_HDRS) $(LIBDIR)/libnetc.so
	@mkdir -p diag
	$(HIPCC) $(HIPFLAGS) -DNETC_ENC_DIAG_NOFIX -shared -o $@ $(GPU_SRCS) -L$(LIBDIR) -lnetc -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'
tools/libscan_k1exp.so: $(GPU_SRCS) $(GPU_HDRS) $(LIBDIR)/libnetc.so
	$(HIPCC) $(HIPFLAGS) -DNETC_SCAN_K1_EXP -shared -o $@ $(GPU_SRCS) -L$(LIBDIR) -lnetc -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'

# ASan + UBSan over the host C (the reference had two heap overflows on this
# path, B1 src/ws/common.c:100 and B6 :306-315; this proves the rebuilt parser has none).
# The instrumented libraries go to build/asan/; Python itself is not instrumented, so the
# sanitizer runtimes are preloaded and leak checking is off (the interpreter's own).
ASAN_FLAGS := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined
ASAN_TESTS := tests/test_host_framing.py tests/test_mask_cpu.py tests/test_oracle.py tests/test_scan_oracle.py tests/test_scan_host.py \
              tests/test_utf8_oracle.py tests/test_route.py
build/asan/libnetc.so: $(HOST_SRCS) $(HOST_HDRS)
	@mkdir -p build/asan
	$(CC) $(ASAN_FLAGS) -Wall -fPIC -std=gnu11 -shared -o $@ $(HOST_SRCS) -lpthread -ldl
build/asan/liboracle.so: oracle/ws_oracle.c
	@mkdir -p build/asan
	$(CC) $(ASAN_FLAGS) -Wall -fPIC -shared -o $@ $<
asan: build/asan/libnetc.so build/asan/liboracle.so oracle
	NETC_HOST_LIB=build/asan/libnetc.so NETC_ORACLE_LIB=build/asan/liboracle.so \
	LD_PRELOAD="$$($(CC) -print-file-name=libasan.so) $$($(CC) -print-file-name=libubsan.so)" \
	ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
	python3 -m pytest -q -m "not gpu" -p no:cacheprovider $(ASAN_TESTS)
