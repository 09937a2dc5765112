"""ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle/ws_oracle.c, oracle/ref_harness.c)."""
