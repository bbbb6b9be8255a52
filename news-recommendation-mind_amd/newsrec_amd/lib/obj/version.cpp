extern "C" const char* nr_build_hash(void) { return "3f09500434c8ddd3"; }
