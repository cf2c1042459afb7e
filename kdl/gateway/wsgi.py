"""WSGI entry for gunicorn: ``gunicorn --bind 0.0.0.0:9696 kdl.gateway.wsgi:app``
(the reference runs ``gunicorn --bind 0.0.0.0:9696 model_server:app``,
`gateway.dockerfile:17`)."""
from .app import create_app

app = create_app()
