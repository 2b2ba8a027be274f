"""Reference-named API modules (RewardModel, ObservationSpaces, ActionSpaces)."""
