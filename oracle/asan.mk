# make ASAN=1 (included by Makefile): the oracle restatement under AddressSanitizer +
# UBSan, driven by asan_check.c over every entry point on small shapes.
SAN = -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all

asan: _ref/asan_check

_ref/asan_check: asan_check.c asw_oracle.c srgb_table.h
	@mkdir -p _ref
	$(CC) -std=c11 -Wall -fopenmp -ffp-contract=off $(SAN) -o $@ asan_check.c asw_oracle.c -lm

.PHONY: asan
