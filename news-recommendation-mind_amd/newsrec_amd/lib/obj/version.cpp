extern "C" const char* nr_build_hash(void) { return "4069e3e6178bd802"; }
