# csrc/knn.hip built without SLP vectorisation (no v_pk_*_f32): is the packed f32 form the trigger?
REPL = [("build_native.py", 'EXTRA_FLAGS = {"cost_volume.hip": ["-fno-slp-vectorize"]}',
         'EXTRA_FLAGS = {"cost_volume.hip": ["-fno-slp-vectorize"], "knn.hip": ["-fno-slp-vectorize"]}')]
