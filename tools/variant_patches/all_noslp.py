# every source without SLP vectorisation
REPL = [("build_native.py", '"-ffp-contract=off",            # every fma the parity contract needs is explicit',
         '"-ffp-contract=off",            # every fma the parity contract needs is explicit\n    "-fno-slp-vectorize",')]
