# oracle/san.mk -- TEST INFRASTRUCTURE ONLY: the oracle under AddressSanitizer + UBSan (host code,
# gcc; no GPU code is involved).  make -C oracle -f san.mk  ->  _san/oracle_san
CC ?= gcc
HERE := $(dir $(abspath $(lastword $(MAKEFILE_LIST))))

$(HERE)_san/oracle_san: $(HERE)inflate_oracle.c $(HERE)sanitize_main.c
	mkdir -p $(HERE)_san
	$(CC) -O1 -g -std=c11 -Wall -Wextra -fsanitize=address,undefined -fno-sanitize-recover=all \
	    -fno-omit-frame-pointer -o $@ $^
