"""Drop-in package mirroring the reference's utils/ (agent_api, kafka_utils, st_functions)."""
