# Repository-level targets (the build itself is __graft_entry__.build(): solvempc_amd/csrc, oracle, tests/cpp).
#   make sanitize : ASan + UBSan builds of the CPU checker (oracle/) and of the C++ host side
#                   (solvempc_amd/cpp via tests/cpp/from_json_check), then the CPU tests that exercise them
#                   (tests/test_oracle.py, tests/test_cpp_surface.py) on those builds, libasan preloaded into
#                   the Python process.  Any ASan report or UBSan runtime error aborts the test (non-zero exit).
ASAN_RT := $(shell gcc -print-file-name=libasan.so)

sanitize:
	$(MAKE) -C oracle -s sanitize
	$(MAKE) -C tests/cpp -s sanitize
	LD_PRELOAD=$(ASAN_RT) ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
	ORACLE_LIB=$(CURDIR)/oracle/liboracle_san.so FROM_JSON_CHECK=$(CURDIR)/tests/cpp/build/from_json_check_san \
	python -m pytest tests/test_oracle.py tests/test_cpp_surface.py -q -m "not gpu" -p no:cacheprovider

.PHONY: sanitize
