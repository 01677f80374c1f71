"""TEST INFRASTRUCTURE ONLY — CPU oracle of the reference mastering chain (see mastering_oracle.py)."""
