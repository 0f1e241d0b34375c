REPL = [("csrc/weightnet.hip", "constexpr int kBwdGrid = 512;", "constexpr int kBwdGrid = 2048;")]
