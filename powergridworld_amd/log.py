"""gridworld/log.py:1-8 equivalent: the "default" logger at INFO."""
import logging

logging.basicConfig(format='[%(levelname)s] %(filename)s:%(lineno)d: %(message)s',
                    level=logging.INFO)
logger = logging.getLogger("default")
