# make ASAN=1 (included by Makefile): host-only AddressSanitizer + UBSan builds of the
# CLI and the PNG tool (SURVEY §5 "Race detection / sanitizers"), next to the normal
# binaries.  g++ only: no device code is compiled with a sanitizer.
SAN = -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all

asan: ../asw_stereo_asan ../png_tool_asan

../asw_stereo_asan: asw_stereo.cpp png_io.cpp png_io.h ../../include/asw.h ../libasw_hip.so
	$(CXX) -std=c++17 -Wall -I../../include $(SAN) -o $@ asw_stereo.cpp png_io.cpp -L$(LIBDIR) -lasw_hip -lz -Wl,-rpath,'$$ORIGIN'

../png_tool_asan: png_tool.cpp png_io.cpp png_io.h
	$(CXX) -std=c++17 -Wall $(SAN) -o $@ png_tool.cpp png_io.cpp -lz

.PHONY: asan
