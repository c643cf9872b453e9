"""CPU oracle — test infrastructure only (see ctr_oracle.py's header)."""
