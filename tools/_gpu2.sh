bash tools/ab_variants.sh lib lib_r2 lib_kc4 && KRE=stack4_kernel bash tools/sq_stack.sh
