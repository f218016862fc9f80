"""gluon/rnn (being implemented)."""
