extern "C" const char* nr_build_hash(void) { return "c87863d217cf7e0c"; }
