"""CPU oracle package -- test infrastructure only (see oracle.h)."""
