"""Auxiliary subsystems: logging, profiling, reports, saved-model I/O."""
