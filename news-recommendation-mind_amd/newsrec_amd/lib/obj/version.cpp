extern "C" const char* nr_build_hash(void) { return "a4fdf88e0055dd65"; }
