#!/bin/bash
# gemm3 epilogue stores plain (abso/lib_A.so) vs non-temporal (abso/lib_N.so, built with
# -DSRNN_G3_NT_STORE=1): same-box alternation of the bench's TBPTT step at 512 / 64 rows
set -e
TAG=r06nt COMBOS="A: N:" ROUNDS=2 LAST=A SITES="'mlp_da1_gemm','mlp_da2_gemm','mlp_dw_hid_gemm','dtab_scatter'" bash tools/r05_combo.sh > gpurun_out/r06nt_combo.txt 2>&1
echo ok
