"""No source change: a variant that differs only in compiler flags
(tools/build_variant.py NAME tools/variant_nop.py FILE.hip=FLAG ...)."""
