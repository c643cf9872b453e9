"""Counterparts of the reference's ``src/main`` drivers (the iPinYou day-split variants)."""
