"""CPU oracle for parity tests (TEST INFRASTRUCTURE ONLY; see velocity_ref.py header)."""
