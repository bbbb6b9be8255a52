extern "C" const char* nr_build_hash(void) { return "70278c44347837a4"; }
