"""REST surface of the brute-force path: the reference's
/vectors routes served from the MI355X store (api/routes/vectors.py)."""
