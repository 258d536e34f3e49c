"""RLlib utilities: schedules, replay buffers."""
