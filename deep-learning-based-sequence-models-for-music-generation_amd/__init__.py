"""midiseq — MI355X-native symbolic-music sequence-model engine."""
