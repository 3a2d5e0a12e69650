"""Small process utilities shared by the daemons."""
