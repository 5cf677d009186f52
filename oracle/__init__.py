"""Test infrastructure only: the CPU checker of the MI355X GICP engine (see gicp_oracle.py)."""
