extern "C" const char* nr_build_hash(void) { return "1a3fe6a1a1ec32bd"; }
